/* Exhaustive check of the glibc-exact sinf/cosf/expf restatements used by the
 * HIP kernels (surf-path-tracer_amd/csrc/device/surf_math.h) against this
 * machine's glibc.  Build: gcc -O2 -ffp-contract=off -I... tools/verify_libm.c -lm
 * Runtime ~40 s.  Used once per glibc/CPU change; tests/ run a sampled version. */
#include <stdio.h>
#include <string.h>
#include <stdint.h>
#include <math.h>
#include "device/surf_math.h"
#include <stdlib.h>
int main(int argc, char** argv) {
    /* optional stride: check every k-th float (tests use a quick stride) */
    const uint32_t step = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 10) : 1u;
    long bad = 0, n = 0; uint32_t hi; float lim;
    lim = 6.3f; memcpy(&hi, &lim, 4);
    for (uint32_t u = 0; u <= hi; u += step) { float f; memcpy(&f, &u, 4);
        float a = sinf(f), b = surfdev::gSinf(f), c = cosf(f), d = surfdev::gCosf(f);
        bad += memcmp(&a, &b, 4) != 0; bad += memcmp(&c, &d, 4) != 0; n += 2; }
    printf("sin/cos [0,6.3]: %ld checks, %ld mismatches\n", n, bad);
    long bad2 = 0, n2 = 0; lim = -110.0f; memcpy(&hi, &lim, 4);
    for (uint32_t u = 0x80000000u; u <= hi; u += step) { float f; memcpy(&f, &u, 4);
        float a = expf(f), b = surfdev::gExpf(f); bad2 += memcmp(&a, &b, 4) != 0; n2++; }
    printf("exp [-110,0]: %ld checks, %ld mismatches\n", n2, bad2);
    return (bad || bad2) ? 1 : 0;
}
