/*
 * render_indoor.cpp -- headless equivalent of the reference's main.cpp GPU loop
 * (sources/main.cpp:141-149 camera, :161-346 scene, :360-442 render loop),
 * written against the drop-in C++ API (include/surf/surf_host.hpp): the scene,
 * BVHs, camera and WaveFrontRenderer are built exactly as the reference's
 * application builds them, with RenderContext holding a HIP device instead of
 * a Vulkan context and no UIManager.
 *
 * usage: render_indoor ASSETS_DIR WIDTH HEIGHT FRAMES OUT.(ppm|png) [--lumen] [--spp N]
 * (--spp: config().samplesPerFrame, the UI's 1..24 slider, ui_manager.cpp:103 /
 * main.cpp:415; a frame's samples continue one RNG stream, renderer.cpp:169-181)
 * Prints the reference's per-frame line (ms, Mrays/s, samples, Lumen; the
 * energy only with --lumen, the reference's WF_LUMEN_OUTPUT, which drains the
 * stream every frame), then one JSON line with the loop's wall time including
 * the final drain, and writes the image as the reference presents it: the RGBA8 finalize image
 * (wavefront_finalize.comp) through fs_quad.frag's sqrt gamma, 8 bits per
 * channel (displayRGBA8), as PPM or PNG by extension.
 */
#include "surf/surf_host.hpp"
#include "indoor_scene.hpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

using namespace surf;

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s ASSETS_DIR WIDTH HEIGHT FRAMES OUT.(ppm|png) [--lumen] [--spp N]\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1];
    const U32 W = (U32)std::atoi(argv[2]), H = (U32)std::atoi(argv[3]), frames = (U32)std::atoi(argv[4]);
    bool lumen = false;
    U32 spp = 1;
    for (int a = 6; a < argc; ++a) {
        const std::string opt = argv[a];
        if (opt == "--lumen") lumen = true;
        else if (opt == "--spp" && a + 1 < argc) spp = (U32)std::max(1, std::atoi(argv[++a]));
        else { std::fprintf(stderr, "unknown option %s\n", opt.c_str()); return 2; }
    }
    try {
        RenderContext context;            /* HIP device 0 */
        Camera worldCam = indoorCamera(W, H);
        IndoorScene indoor(&context, dir);          /* main.cpp:161-346 */
        GPUScene& scene = *indoor.scene;

        RendererConfig config;            /* samplesPerFrame 1 (ui_manager.h:26) unless --spp, unbounded + RR */
        config.samplesPerFrame = spp;
        config.lumenOutput = lumen;
        WaveFrontRenderer renderer(&context, nullptr, config, FramebufferSize{W, H}, worldCam, scene);

        const auto tLoop = std::chrono::steady_clock::now();
        for (U32 f = 0; f < frames; ++f) {
            const auto t0 = std::chrono::steady_clock::now();
            renderer.render(0.0f);        /* returns once the frame's samples are issued (lumenOutput: frameInfo() drains) */
            const FrameInstrumentationData& info = renderer.frameInfo();
            const auto t1 = std::chrono::steady_clock::now();
            const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
            /* main.cpp:431-442's line.  Without --lumen, render() returns once the
             * frame is issued, so `ms` is the ISSUE latency of the call, not a
             * frame time; the rate printed is samples ISSUED so far over the
             * loop's wall time (frames still in flight included, so it reads
             * high until the drain); the finished-sample rate of the loop is the
             * final JSON line's mrays_per_s */
            const double loopSoFar = std::chrono::duration<double, std::milli>(t1 - tLoop).count();
            std::printf("%08.2fms issue (%05.1f calls/s) - %08.2fMrays/s issued avg - %05u samples (%u spp) - %010.2f Lumen\n", ms,
                        1000.0 / ms, (double)W * H * renderer.config().samplesPerFrame * (f + 1) / loopSoFar / 1000.0,
                        info.totalSamples, renderer.config().samplesPerFrame, info.energy);
        }

        renderer.synchronize();           /* every frame accumulated */
        const double loopMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tLoop).count();
        std::printf("{\"frames\": %u, \"samples_per_frame\": %u, \"width\": %u, \"height\": %u, \"loop_ms\": %.3f, \"mrays_per_s\": %.3f, "
                    "\"lumen_output\": %s}\n",
                    frames, spp, W, H, loopMs, (double)W * H * frames * spp / loopMs / 1000.0, config.lumenOutput ? "true" : "false");
        const std::vector<U32> img = renderer.displayRGBA8();
        const std::string path = argv[5];
        const bool png = path.size() > 4 && path.compare(path.size() - 4, 4, ".png") == 0;
        const int rc = png ? surf_write_png(path.c_str(), W, H, img.data()) : surf_write_ppm(path.c_str(), W, H, img.data());
        if (rc != SURF_OK) { std::fprintf(stderr, "cannot write %s\n", path.c_str()); return 1; }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "render_indoor: %s\n", e.what());
        return 1;
    }
    return 0;
}
