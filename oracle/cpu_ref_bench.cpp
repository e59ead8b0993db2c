/*
 * oracle/cpu_ref_bench.cpp -- CLI around the CPU oracle: the timed CPU baseline
 * (bench.py cpu_baseline leg) and a PFM writer for eyeballing renders.
 * TEST INFRASTRUCTURE ONLY (see cpu_ref.h).
 *
 * usage: cpu_ref_bench [options] ASSETS W H FRAMES [ROW_BEGIN ROW_END [MAX_SEG [THREADS [OUT.pfm]]]]
 *   --cutoff       end paths whose throughput fell below FLT_MIN (orc_set_zero_cutoff),
 *                  as the GPU renderer does by default
 *   --variant N    scene variant (1 = C5 deep scene)
 *   --first F      first frame index (frame f seeded initSeed(p + 1799 (F + f)))
 *   --row-step S   render rows ROW_BEGIN, ROW_BEGIN + S, ... < ROW_END (a spread sample)
 *   --dump PATH    write the float RGBA accumulator of the rendered rows (raw f32,
 *                  rows in order) for a bit-exact comparison with the GPU's
 * prints one JSON line: samples, seconds, mrays_per_s, threads, event counts.
 * The row loop is renderer.cpp:163's `omp parallel for schedule(dynamic)`.
 */
#include "cpu_ref.h"
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include <omp.h>

int main(int argc, char** argv) {
    int cutoff = 0, variant = 0;
    uint32_t first = 0, step = 1;
    const char* dump = nullptr;
    for (;;) {
        const std::string a = argc > 1 ? argv[1] : "";
        if (a == "--cutoff") {
            cutoff = 1;
            orc_set_zero_cutoff(1);
            ++argv; --argc;
        } else if (argc > 2 && (a == "--variant" || a == "--first" || a == "--row-step" || a == "--dump")) {
            if (a == "--variant") variant = atoi(argv[2]);
            else if (a == "--first") first = (uint32_t)strtoul(argv[2], nullptr, 10);
            else if (a == "--row-step") step = (uint32_t)strtoul(argv[2], nullptr, 10);
            else dump = argv[2];
            argv += 2; argc -= 2;
        } else {
            break;
        }
    }
    if (argc < 5) { fprintf(stderr, "usage: %s [options] ASSETS W H FRAMES [ROW_BEGIN ROW_END [MAX_SEG [THREADS [OUT.pfm]]]]\n", argv[0]); return 2; }
    const char* assets = argv[1];
    uint32_t W = (uint32_t)atoi(argv[2]), H = (uint32_t)atoi(argv[3]), F = (uint32_t)atoi(argv[4]);
    uint32_t r0 = argc > 6 ? (uint32_t)atoi(argv[5]) : 0, r1 = argc > 6 ? (uint32_t)atoi(argv[6]) : H;
    uint32_t maxSeg = argc > 7 ? (uint32_t)atoi(argv[7]) : 0;
    int threads = argc > 8 ? atoi(argv[8]) : 0;
    const char* out = argc > 9 ? argv[9] : nullptr;
    if (r1 > H || r0 >= r1 || W == 0 || F == 0 || step == 0) { fprintf(stderr, "bad arguments\n"); return 2; }
    orc_scene* s = orc_scene_create(assets, variant);
    if (!s) return 1;
    std::vector<uint32_t> rows;
    for (uint32_t y = r0; y < r1; y += step) rows.push_back(y);
    std::vector<float> acc(rows.size() * W * 4, 0.0f);
    orc_counters c;
    double sec = orc_render_rows(s, W, H, rows.data(), (uint32_t)rows.size(), first, F, maxSeg, threads, acc.data(), &c);
    int used = threads > 0 ? threads : omp_get_max_threads();
    printf("{\"samples\": %llu, \"seconds\": %.6f, \"mrays_per_s\": %.4f, \"threads\": %d, \"rows\": %zu, "
           "\"n_ext\": %llu, \"n_hit\": %llu, \"n_cont\": %llu, \"n_shadow\": %llu, \"n_acc\": %llu, \"n_unocc\": %llu, \"max_segments\": %llu, \"cutoff\": %d}\n",
           (unsigned long long)c.samples, sec, (double)c.samples / sec / 1e6, used, rows.size(),
           (unsigned long long)c.n_ext, (unsigned long long)c.n_hit, (unsigned long long)c.n_cont,
           (unsigned long long)c.n_shadow, (unsigned long long)c.n_acc, (unsigned long long)c.n_unocc,
           (unsigned long long)c.max_segments, cutoff);
    if (dump) {
        FILE* f = fopen(dump, "wb");
        if (!f || fwrite(acc.data(), sizeof(float), acc.size(), f) != acc.size()) { fprintf(stderr, "cannot write %s\n", dump); return 1; }
        fclose(f);
    }
    if (out) {
        FILE* f = fopen(out, "wb");
        if (f) {
            const uint32_t n = (uint32_t)rows.size();
            fprintf(f, "PF\n%u %u\n-1.0\n", W, n);
            for (int64_t y = (int64_t)n - 1; y >= 0; --y)
                for (uint32_t x = 0; x < W; ++x) { const float* a = &acc[4 * ((size_t)y * W + x)]; float rgb[3] = {a[0] / F, a[1] / F, a[2] / F}; fwrite(rgb, 4, 3, f); }
            fclose(f);
        }
    }
    orc_scene_destroy(s);
    return 0;
}
