/*
 * renderer_host.cpp -- WaveFrontRenderer (headers/renderer.h:207-436) on top of
 * the C-ABI.  render() keeps the reference's CPU frame semantics: every call
 * adds config().samplesPerFrame samples per pixel, seeded once per frame from
 * the running sample count (renderer.cpp:169) and run in sequence on that one
 * RNG stream (renderer.cpp:171-181), and camera state is re-read per frame
 * (renderer.cpp:972-979).  render() returns once the frame's samples are
 * issued: consecutive frames form one sample stream on the device (no
 * per-frame drain); reads (accumulator, images, frameInfo() with lumenOutput)
 * drain it.  Errors throw std::runtime_error (the reference aborts through
 * VK_CHECK).
 */
#include "surf/surf_host.hpp"

#include <stdexcept>
#include <string>

namespace surf {

namespace {
void check(int rc, surf_ctx* ctx, const char* what) {
    if (rc != SURF_OK) throw std::runtime_error(std::string(what) + ": " + surf_last_error(ctx));
}
}  // namespace

WaveFrontRenderer::WaveFrontRenderer(RenderContext* context, UIManager* /*uiManager*/, RendererConfig config,
                                     FramebufferSize resolution, Camera& camera, GPUScene& scene)
    : m_config(config), m_resolution(resolution), m_camera(camera), m_scene(scene) {
    const int dev = context ? context->hipDevice : 0;
    check(surf_create(dev, resolution.width, resolution.height, 0, resolution.height, &m_ctx), nullptr, "surf_create");
    const surf_scene_desc desc = scene.descriptor();
    check(surf_upload_scene(m_ctx, &desc), m_ctx, "surf_upload_scene");
    m_sceneGeneration = scene.generation();
}

WaveFrontRenderer::~WaveFrontRenderer() { surf_destroy(m_ctx); }

void WaveFrontRenderer::clearAccumulator() {
    check(surf_clear_accumulator(m_ctx), m_ctx, "surf_clear_accumulator");
    m_totalSamples = 0;
    m_frameInfo = FrameInstrumentationData{};
    m_energyStale = false;
}

void WaveFrontRenderer::render(F32 /*deltaTime*/) {
    if (m_scene.generation() != m_sceneGeneration) {
        /* GPUScene::update (scene.cpp:267-282) re-uploads the instance records,
         * TLAS indices and TLAS nodes; geometry and BLASes stay resident */
        const surf_scene_desc desc = m_scene.descriptor();
        if (surf_update_instances(m_ctx, desc.instances, desc.instance_count, desc.tlas_indices, desc.tlas_nodes,
                                  desc.tlas_node_count, desc.lights, desc.light_count) != SURF_OK)
            check(surf_upload_scene(m_ctx, &desc), m_ctx, "surf_upload_scene");
        m_sceneGeneration = m_scene.generation();
    }
    const CameraUBO ubo = m_camera.toUBO();
    check(surf_set_camera(m_ctx, &ubo), m_ctx, "surf_set_camera");
    /* one frame of samplesPerFrame samples, seeded from the running sample
     * count, its samples chaining their RNG state (renderer.cpp:160-188) */
    const U32 spp = m_config.samplesPerFrame ? m_config.samplesPerFrame : 1u;
    check(surf_render(m_ctx, 1, m_totalSamples, m_config.maxSegments, spp), m_ctx, "surf_render");
    m_totalSamples += spp;
    m_frameInfo.totalSamples = m_totalSamples;
    m_energyStale = true;       /* render() itself never waits for the stream (no per-frame drain) */
}

/* The reference computes the Lumen energy only with WF_LUMEN_OUTPUT
 * (renderer.cpp:31, off by default; :955-969), from the accumulator of the
 * frames rendered so far.  Here it is computed when asked for: the energy
 * needs every rendered frame accumulated, which drains the sample stream. */
const FrameInstrumentationData& WaveFrontRenderer::frameInfo() {
    if (m_config.lumenOutput && m_energyStale && m_totalSamples) {
        surf_stats st;
        check(surf_get_stats(m_ctx, &st), m_ctx, "surf_get_stats");
        m_frameInfo.energy = st.energy;
        m_energyStale = false;
    }
    return m_frameInfo;
}

void WaveFrontRenderer::synchronize() { check(surf_synchronize(m_ctx), m_ctx, "surf_synchronize"); }

std::vector<F32> WaveFrontRenderer::readAccumulator() {
    std::vector<F32> out((size_t)m_resolution.width * m_resolution.height * 4);
    check(surf_read_accumulator(m_ctx, out.data()), m_ctx, "surf_read_accumulator");
    return out;
}

std::vector<U32> WaveFrontRenderer::finalizeRGBA8() {
    std::vector<U32> out((size_t)m_resolution.width * m_resolution.height);
    check(surf_finalize_rgba8(m_ctx, out.data()), m_ctx, "surf_finalize_rgba8");
    return out;
}

std::vector<U32> WaveFrontRenderer::displayRGBA8() {
    std::vector<U32> out((size_t)m_resolution.width * m_resolution.height);
    check(surf_display_rgba8(m_ctx, out.data()), m_ctx, "surf_display_rgba8");
    return out;
}

}  // namespace surf
