#!/bin/bash
# Per-function register / scratch usage of the detection kernels (developer tool).
cd /tmp && rm -rf regs_tmp && mkdir regs_tmp && cd regs_tmp
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I/root/repo/include ${KFLAGS} -c /root/repo/lcmap-firebird_amd/csrc/ccd_kernels.hip -o k.o -save-temps 2>&1 | grep -E "error" 
awk '/^_Z[A-Za-z0-9_]*:/{name=$1} /; NumVgprs:/{v=$3} /; NumAgprs:/{a=$3} /; ScratchSize:/{printf "%-60s vgpr %4s agpr %4s scratch %4s\n", substr(name,1,60), v, a, $3}' ccd_kernels-hip-amdgcn-amd-amdhsa-gfx950.s
grep -E "\.vgpr_count|\.sgpr_count|\.name:|private_segment_fixed_size" ccd_kernels-hip-amdgcn-amd-amdhsa-gfx950.s | grep -A3 -B1 "ccd_detect" | head -8
