/*
 * render_indoor_mgpu.cpp -- the reference's scene rendered on several GPUs of
 * one node from a C++ application: the frame is split into
 * pixel-row shards (surf_create_sharded: interleaved blocks of ROW_BLOCK rows,
 * block b on GPU b % N), each GPU renders its rows on its own host thread with
 * no communication, and one RCCL gather (libsurf_mgpu: ncclCommInitAll, one
 * ncclGather per rank in one group) brings the float accumulators to GPU 0,
 * whose rows are un-permuted into the frame.  The assembled frame equals the
 * one-GPU frame bit for bit (every sample depends only on its pixel and its
 * sample index).
 *
 * usage: render_indoor_mgpu ASSETS_DIR WIDTH HEIGHT FRAMES OUT.(ppm|png)
 *                           [--gpus N] [--row-block B] [--spp K]
 * Prints one JSON line: render and gather wall times, Mrays/s of the whole job.
 */
#include "surf/surf_host.hpp"
#include "surf_mgpu.h"
#include "indoor_scene.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <stdexcept>
#include <thread>
#include <vector>

using namespace surf;

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s ASSETS_DIR WIDTH HEIGHT FRAMES OUT.(ppm|png) [--gpus N] [--row-block B] [--spp K]\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1];
    const U32 W = (U32)std::atoi(argv[2]), H = (U32)std::atoi(argv[3]), frames = (U32)std::atoi(argv[4]);
    int gpus = 0;
    U32 rowBlock = 1, spp = 1;
    for (int a = 6; a < argc; ++a) {
        const std::string opt = argv[a];
        if (opt == "--gpus" && a + 1 < argc) gpus = std::atoi(argv[++a]);
        else if (opt == "--row-block" && a + 1 < argc) rowBlock = (U32)std::atoi(argv[++a]);
        else if (opt == "--spp" && a + 1 < argc) spp = (U32)std::max(1, std::atoi(argv[++a]));
        else { std::fprintf(stderr, "unknown option %s\n", opt.c_str()); return 2; }
    }
    int devices = 0;
    if (surf_device_count(&devices) != SURF_OK || devices == 0) { std::fprintf(stderr, "no HIP device\n"); return 1; }
    if (gpus <= 0) gpus = devices;
    if (gpus > devices) { std::fprintf(stderr, "%d GPUs requested, %d present\n", gpus, devices); return 1; }
    try {
        RenderContext context;                        /* the scene is built once on the host */
        IndoorScene indoor(&context, dir);
        const surf_scene_desc desc = indoor.scene->descriptor();
        const CameraUBO ubo = indoorCamera(W, H).toUBO();

        /* one shard context per GPU: the scene replicated, the rows split */
        std::vector<surf_ctx*> shards(gpus, nullptr);
        auto check = [&](int rc, surf_ctx* c, const char* what) {
            if (rc != SURF_OK) throw std::runtime_error(std::string(what) + ": " + surf_last_error(c));
        };
        for (int g = 0; g < gpus; ++g) {
            check(surf_create_sharded(g, W, H, (U32)g, (U32)gpus, rowBlock, &shards[g]), nullptr, "surf_create_sharded");
            check(surf_upload_scene(shards[g], &desc), shards[g], "surf_upload_scene");
            check(surf_set_camera(shards[g], &ubo), shards[g], "surf_set_camera");
        }
        std::vector<surf_mgpu*> ranks(gpus, nullptr);
        if (surf_mgpu_create_all(shards.data(), (U32)gpus, W, H, rowBlock, ranks.data()) != SURF_OK)
            throw std::runtime_error(std::string("surf_mgpu_create_all: ") + surf_mgpu_last_error());

        /* every GPU renders its rows on its own thread, then drains */
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<int> rcs(gpus, SURF_OK);
        std::vector<std::thread> threads;
        for (int g = 0; g < gpus; ++g)
            threads.emplace_back([&, g] {
                rcs[g] = surf_render(shards[g], frames, 0, 0, spp);
                if (rcs[g] == SURF_OK) rcs[g] = surf_synchronize(shards[g]);
            });
        for (auto& t : threads) t.join();
        for (int g = 0; g < gpus; ++g) check(rcs[g], shards[g], "surf_render");
        const auto t1 = std::chrono::steady_clock::now();
        std::vector<F32> frame((size_t)W * H * 4, 0.0f);
        if (surf_mgpu_gather_all(ranks.data(), (U32)gpus, frame.data()) != SURF_OK)
            throw std::runtime_error(std::string("surf_mgpu_gather_all: ") + surf_mgpu_last_error());
        const auto t2 = std::chrono::steady_clock::now();

        const double renderMs = std::chrono::duration<double, std::milli>(t1 - t0).count();
        const double gatherMs = std::chrono::duration<double, std::milli>(t2 - t1).count();
        const double samples = (double)W * H * frames * spp;
        std::printf("{\"gpus\": %d, \"row_block\": %u, \"frames\": %u, \"samples_per_frame\": %u, \"width\": %u, \"height\": %u, "
                    "\"render_ms\": %.3f, \"gather_ms\": %.3f, \"mrays_per_s\": %.3f}\n",
                    gpus, rowBlock, frames, spp, W, H, renderMs, gatherMs, samples / (renderMs + gatherMs) / 1000.0);

        std::vector<U32> img((size_t)W * H);
        check(surf_pack_rgba8(frame.data(), W * H, 1.0f / (float)(frames * spp), 1, img.data()), nullptr, "surf_pack_rgba8");
        const std::string path = argv[5];
        const bool png = path.size() > 4 && path.compare(path.size() - 4, 4, ".png") == 0;
        const int rc = png ? surf_write_png(path.c_str(), W, H, img.data()) : surf_write_ppm(path.c_str(), W, H, img.data());
        for (int g = 0; g < gpus; ++g) { surf_mgpu_destroy(ranks[g]); surf_destroy(shards[g]); }
        if (rc != SURF_OK) { std::fprintf(stderr, "cannot write %s\n", path.c_str()); return 1; }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "render_indoor_mgpu: %s\n", e.what());
        return 1;
    }
    return 0;
}
