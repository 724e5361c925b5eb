/*
 * libm_check.c — TEST INFRASTRUCTURE: checks llamacog_amd/csrc/libm_exact.h (the device
 * restatement of glibc's FMA-build expf / sinf / cosf) against this host's libm, bit for bit.
 *
 *   libm_check <func 0=expf 1=sinf 2=cosf> <lo> <hi> <stride>
 *
 * walks every `stride`-th float bit pattern in [lo, hi] (both finite, same sign) and prints
 * the number of inputs checked and of mismatches (plus the first few).  Built by
 * oracle/Makefile with -ffp-contract=off so that only the explicit fma() calls fuse.
 */
#include <stdio.h>
#include <stdlib.h>
#include "../llamacog_amd/csrc/libm_exact.h"

static float ref(int f, float x) { return f == 0 ? expf(x) : (f == 1 ? sinf(x) : cosf(x)); }
static float mine(int f, float x) { return f == 0 ? lx_expf(x) : (f == 1 ? lx_sinf(x) : lx_cosf(x)); }

int main(int argc, char ** argv) {
    if (argc < 5) return 2;
    const int f = atoi(argv[1]);
    const float lo = strtof(argv[2], NULL), hi = strtof(argv[3], NULL);
    const uint32_t stride = (uint32_t) strtoul(argv[4], NULL, 10);
    uint32_t a = lx_asuint(lo), b = lx_asuint(hi);
    if (a > b) { uint32_t t = a; a = b; b = t; }
    unsigned long long n = 0, bad = 0;
    for (uint64_t u = a; u <= b; u += stride) {
        float x;
        const uint32_t v = (uint32_t) u;
        memcpy(&x, &v, 4);
        const float r = ref(f, x), m = mine(f, x);
        ++n;
        if (lx_asuint(r) != lx_asuint(m)) {
            if (bad < 5) printf("mismatch f=%d x=%a ref=%a mine=%a\n", f, x, r, m);
            ++bad;
        }
    }
    printf("checked %llu mismatches %llu\n", n, bad);
    return bad != 0;
}
