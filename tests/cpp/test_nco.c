/* TEST INFRASTRUCTURE: the front-end kernels rebuild oscillatorTable (ofdm-processor.cpp:
 * 79-81) from three small factor tables (dab_kernels.h, NCO_*; nco_value in dab_device.h)
 * instead of reading the 16 MB table.  This restates that double-precision formula
 * (IEEE fma and mul are exact to restate) on the product's own factor tables and checks
 * it against the oracle's oscillatorTable at all 2048000 indices.  No GPU needed. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include "dabgpu.h"
#include "dab_oracle.h"

typedef struct { double r, i; } cd;
static cd mul(cd a, cd b) {
    cd o;
    const double p = a.i * b.i, q = a.i * b.r;
    o.r = fma(a.r, b.r, -p);
    o.i = fma(a.r, b.i, q);
    return o;
}

int main(void) {
    static cd tab[384];
    if (dabgpu_host_table(DABGPU_TABLE_NCO, tab, sizeof tab) != 0) { printf("no NCO table\n"); return 2; }
    static float osc[2 * 2048000];
    if (dabgpu_host_table(DABGPU_TABLE_OSC, osc, sizeof osc) != 0) { printf("no OSC table\n"); return 2; }
    long bad = 0, bad_tab = 0;
    for (int32_t t = 0; t < 2048000; t++) {
        const uint32_t a = (uint32_t)t / 16000u, r = (uint32_t)t - a * 16000u;
        const cd v = mul(tab[a], mul(tab[128 + (r >> 7)], tab[253 + (r & 127u)]));
        float re, im;
        orc_osc_entry(t, &re, &im);
        bad_tab += memcmp(&osc[2 * t], &re, 4) != 0 || memcmp(&osc[2 * t + 1], &im, 4) != 0;
        const float vr = (float)v.r, vi = (float)v.i;
        if (memcmp(&vr, &re, 4) != 0 || memcmp(&vi, &im, 4) != 0) {
            if (bad < 5) printf("t=%d: %.9g %.9g vs %.9g %.9g\n", t, (float)v.r, (float)v.i, re, im);
            bad++;
        }
    }
    printf("NCO formula: %ld of 2048000 entries differ; product oscillatorTable: %ld differ\n", bad, bad_tab);
    return bad != 0 || bad_tab != 0;
}
