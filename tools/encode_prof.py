#!/usr/bin/env python3
"""Host encoder profile: builds csrc/ccd_encode.c with timers around its two passes (a copy
under the output directory; the product source is not changed) and a driver that encodes two
synthetic 10,000-pixel chips (1421 observations, 13 QA words, 45 % of them dropped by the
'unread' bits), and prints per-pass milliseconds and raw-input GB/s at 1, 3 and 6 threads.

usage: encode_prof.py <out_dir>"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r'''
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <omp.h>
#include "enc_timed.c"
int main(int argc, char **argv) {
  int np = 10000, no = 1421, nc = 2;
  uint16_t pal[13] = {322, 324, 328, 336, 352, 386, 388, 392, 400, 416, 480, 834, 1};
  int16_t *sp[2]; uint16_t *qa[2]; int32_t npx[2] = {np, np}, nob[2] = {no, no};
  uint64_t x = 88172645463325252ull;
  for (int c = 0; c < nc; ++c) {
    sp[c] = malloc((size_t)7 * np * no * 2); qa[c] = malloc((size_t)np * no * 2);
    for (size_t i = 0; i < (size_t)np * no; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; int r = (int)(x % 100); qa[c][i] = r < 55 ? pal[r % 4] : pal[4 + r % 9]; }
    for (size_t i = 0; i < (size_t)7 * np * no; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; sp[c][i] = (int16_t)(x & 4095); }
    for (size_t i = 0; i < (size_t)np * no; ++i) if (qa[c][i] & 1) for (int b = 0; b < 7; ++b) sp[c][(size_t)b * np * no + i] = -9999;
  }
  int64_t cap = ccdgpu_encoded_bound(nc, npx, nob);
  uint8_t *out = malloc(cap);
  const int ths[3] = {1, 3, 6};
  for (int k = 0; k < 3; ++k) {
    double best = 1e9, b1 = 0, b2 = 0;
    for (int rep = 0; rep < 5; ++rep) {
      T1 = T2 = 0; double t = omp_get_wtime();
      ccdgpu_encode_chips(nc, npx, nob, (const int16_t *const *)sp, (const uint16_t *const *)qa, out, cap, ths[k], 1 | 8 | 32, 1);
      t = omp_get_wtime() - t;
      if (t < best) { best = t; b1 = T1; b2 = T2; }
    }
    double raw = (double)nc * np * no * 16;
    printf("threads %d: %.1f ms, %.2f GB/s raw (%.2f per thread); pass1 %.1f ms, pass2 %.1f ms\n", ths[k], best * 1e3, raw / best / 1e9, raw / best / 1e9 / ths[k], b1 * 1e3, b2 * 1e3);
  }
  return 0;
}
'''


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    s = open(os.path.join(ROOT, 'lcmap-firebird_amd', 'csrc', 'ccd_encode.c')).read()
    for a, b in (('#define ENC_HDR 128', 'static double T1, T2;\n#define ENC_HDR 128'),
                 ('    const int vec1 = have_vbmi2();', '    const int vec1 = have_vbmi2();\n    double T0 = omp_get_wtime();'),
                 ('        int bad = 0;  /* (pass 2',
                  '        T1 += omp_get_wtime() - T0; T0 = omp_get_wtime();\n        int bad = 0;  /* (pass 2'),
                 ('        if (miss && !full) continue;',
                  '        T2 += omp_get_wtime() - T0; T0 = omp_get_wtime();\n        if (miss && !full) continue;')):
        assert s.count(a) == 1, a
        s = s.replace(a, b)
    open(os.path.join(out, 'enc_timed.c'), 'w').write(s)
    open(os.path.join(out, 'drv.c'), 'w').write(DRIVER)
    exe = os.path.join(out, 'encode_prof')
    subprocess.run(['gcc', '-O3', '-fopenmp', '-I' + os.path.join(ROOT, 'include'), '-I' + out,
                    os.path.join(out, 'drv.c'), '-o', exe], check=True)
    for blk in ('32', '1'):
        print('CCDGPU_ENCODE_BLOCK=%s' % blk, flush=True)
        subprocess.run([exe], env=dict(os.environ, CCDGPU_ENCODE_BLOCK=blk), check=True)


if __name__ == '__main__':
    main()
