#!/bin/bash
# Developer tool: the w3 detection kernel's assembly into /tmp/regs_tmp/w3.s (after tools/regs.sh).
S=/tmp/regs_tmp/ccd_kernels-hip-amdgcn-amd-amdhsa-gfx950.s
st=$(grep -n "^_ZN12_GLOBAL__N_113ccd_detect_w3Ev:" $S | cut -d: -f1)
en=$(grep -n "^_ZN12_GLOBAL__N_18ccd_prep" $S | cut -d: -f1)
sed -n ${st},${en}p $S > /tmp/regs_tmp/w3.s
