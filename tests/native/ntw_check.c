/* CPU check of the encoder's streaming writer (lcmap-firebird_amd/csrc/ccd_encode.c: ntw_begin /
 * ntw_put / ntw_end, AVX-512F/BW only): random chunk sizes (0..32 values) appended to ranges of
 * random start alignment and length inside a guarded buffer; every range must equal the values
 * appended, and every byte outside it keep its sentinel.  Built and run by tests/test_encode.py. */
#include "../../lcmap-firebird_amd/csrc/ccd_encode.c"

#include <stdio.h>

__attribute__((target("avx512f,avx512bw"))) static int run(unsigned seed) {
    enum { CAP = 1 << 16 };
    static int16_t buf[CAP + 256] __attribute__((aligned(64)));
    static int16_t want[CAP];
    static ntw_t w;
    int16_t src[32];
    unsigned s = seed;
#define RND() (s = s * 1103515245u + 12345u, (s >> 8))
    for (int i = 0; i < CAP + 256; ++i) buf[i] = (int16_t)0x5A5A;
    const int start = 64 + (int)(RND() % 97);            /* element offset: any alignment */
    const int len = (int)(RND() % 3) == 0 ? (int)(RND() % 40) : (int)(RND() % (CAP - 512));
    ntw_begin(&w, buf + start);
    int k = 0;
    while (k < len) {
        int c = (int)(RND() % 33);
        if (c > len - k) c = len - k;
        for (int j = 0; j < 32; ++j) src[j] = (int16_t)(j < c ? RND() : 0x7777);
        for (int j = 0; j < c; ++j) want[k + j] = src[j];
        ntw_put(&w, _mm512_loadu_si512((const void *)src), c);
        k += c;
    }
    ntw_end(&w);
    _mm_sfence();
    for (int i = 0; i < CAP + 256; ++i) {
        const int in = i >= start && i < start + len;
        if (in && buf[i] != want[i - start]) {
            printf("seed %u: value %d of %d (start %d) wrong\n", seed, i - start, len, start);
            return 1;
        }
        if (!in && buf[i] != (int16_t)0x5A5A) {
            printf("seed %u: element %d outside the range [%d, %d) written\n", seed, i, start, start + len);
            return 1;
        }
    }
    return 0;
}

int main(void) {
    if (!__builtin_cpu_supports("avx512f") || !__builtin_cpu_supports("avx512bw")) {
        printf("skip: no AVX-512F/BW\n");
        return 0;
    }
    for (unsigned seed = 1; seed <= 400; ++seed)
        if (run(seed)) return 1;
    printf("ok\n");
    return 0;
}
