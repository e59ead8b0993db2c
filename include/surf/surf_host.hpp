/*
 * surf_host.hpp -- C++ host API of the MI355X wavefront path tracer.
 *
 * Same class names, constructor shapes and semantics as the reference's host
 * API, so a caller of the reference GPU path (main.cpp) switches by swapping
 * includes:
 *   Float2/Float3/Float4 + operators ...... headers/surf_math.h:25-200
 *   Mat4 / translate / scale / rotate ...... glm subset used by main.cpp:204-341, bvh.cpp:486-594
 *   Triangle / TriExtension / Mesh ......... headers/mesh.h:12-75, sources/mesh.cpp
 *   AABB / BvhNode / BvhBLAS ............... headers/bvh.h:12-90, sources/bvh.cpp:17-465
 *   Material ............................... headers/material.h:6-19
 *   GPUInstance / Instance ................. headers/bvh.h:93-147, sources/bvh.cpp:467-594
 *   BvhTLAS ................................ headers/bvh.h:149-193, sources/bvh.cpp:596-993
 *   SceneBackground / GPULightData ......... headers/scene.h:12-71
 *   GPUBatchInfo / GPUBatcher .............. headers/scene.h:73-88, sources/scene.cpp:61-157
 *   GPUScene ............................... headers/scene.h:90-123, sources/scene.cpp:159-282
 *   Camera / CameraUBO ..................... headers/camera.h, sources/camera.cpp
 *   RendererConfig / IRenderer / WaveFrontRenderer ... headers/renderer.h:24-97,207-436
 *
 * Differences, all deliberate: `RenderContext` is a HIP device handle (no
 * Vulkan), the UIManager argument is accepted and ignored (headless), and
 * WaveFrontRenderer adds headless readback (readAccumulator / finalizeRGBA8).
 * Record layouts are byte-identical to the reference (static_asserts below).
 * All GPU work goes through the C-ABI in surf_hip.h.
 */
#pragma once

#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "../surf_hip.h"

namespace surf {

using U32 = uint32_t;
using I32 = int32_t;
using F32 = float;
using SizeType = size_t;

constexpr F32 F32_FAR_AWAY = 1e30f;
constexpr F32 F32_EPSILON = 1e-5f;
constexpr F32 F32_PI = 3.14159265358979323846264f;
constexpr F32 F32_INV_PI = 0.31830988618379067153777f;
constexpr U32 UNSET_INDEX = ~0u;

/* ------------------------------------------------------------ vectors */
struct Float2 {
    F32 x, y;
    Float2() : x(0.0f), y(0.0f) {}
    explicit Float2(F32 s) : x(s), y(s) {}
    Float2(F32 x_, F32 y_) : x(x_), y(y_) {}
};

struct Float3 {
    F32 x, y, z;
    Float3() : x(0.0f), y(0.0f), z(0.0f) {}
    Float3(F32 s) : x(s), y(s), z(s) {}          /* implicit like the reference: F32 * Float3 */
    Float3(F32 x_, F32 y_, F32 z_) : x(x_), y(y_), z(z_) {}
    F32 operator[](SizeType i) const { return i == 0 ? x : (i == 1 ? y : z); }
    F32 dot(const Float3& o) const { return x * o.x + y * o.y + z * o.z; }
    Float3 cross(const Float3& o) const { return Float3(y * o.z - z * o.y, z * o.x - x * o.z, x * o.y - y * o.x); }
    F32 magnitude() const { return sqrtf(dot(*this)); }
    inline Float3 normalize() const;
};
inline Float3 operator+(const Float3& a, const Float3& b) { return Float3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline Float3 operator-(const Float3& a, const Float3& b) { return Float3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline Float3 operator*(const Float3& a, const Float3& b) { return Float3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline Float3 operator/(const Float3& a, const Float3& b) { return Float3(a.x / b.x, a.y / b.y, a.z / b.z); }
inline Float3 operator*(const Float3& a, F32 s) { return Float3(a.x * s, a.y * s, a.z * s); }
inline Float3 operator/(const Float3& a, F32 s) { return Float3(a.x / s, a.y / s, a.z / s); }
inline Float3& operator+=(Float3& a, const Float3& b) { a = a + b; return a; }
inline Float3& operator*=(Float3& a, const Float3& b) { a = a * b; return a; }
inline Float3 Float3::normalize() const { F32 inv = 1.0f / sqrtf(dot(*this)); return *this * inv; }
inline Float3 min(const Float3& a, const Float3& b) { return Float3(a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z); }
inline Float3 max(const Float3& a, const Float3& b) { return Float3(a.x > b.x ? a.x : b.x, a.y > b.y ? a.y : b.y, a.z > b.z ? a.z : b.z); }

struct Float4 {
    F32 x, y, z, w;
    Float4() : x(0), y(0), z(0), w(0) {}
    Float4(F32 x_, F32 y_, F32 z_, F32 w_) : x(x_), y(y_), z(z_), w(w_) {}
    Float4(const Float3& v, F32 w_) : x(v.x), y(v.y), z(v.z), w(w_) {}
};

const Float3 WORLD_FORWARD(0.0f, 0.0f, -1.0f);   /* camera.h:7-9 */
const Float3 WORLD_RIGHT(1.0f, 0.0f, 0.0f);
const Float3 WORLD_UP(0.0f, 1.0f, 0.0f);

/* radians() of surf_math.h:231 (not glm::radians) */
inline F32 radians(F32 deg) { return (deg * F32_PI) * 0.005555555555555f; }

/* ------------------------------------------------------------ Mat4 (glm subset) */
struct Mat4 {
    F32 c[4][4];                         /* column major, glm::mat4 layout */
    explicit Mat4(F32 diag = 1.0f);
    Float4 operator*(const Float4& v) const;
};
Mat4 translate(const Mat4& m, const Float3& v);
Mat4 scale(const Mat4& m, const Float3& v);
Mat4 rotate(const Mat4& m, F32 angle, const Float3& axis);
Mat4 inverse(const Mat4& m);

/* ------------------------------------------------------------ mesh */
struct alignas(16) Triangle {
    alignas(16) Float3 v0;
    alignas(16) Float3 v1;
    alignas(16) Float3 v2;
    alignas(16) Float3 centroid;
    Triangle(Float3 v1, Float3 v0, Float3 v2);   /* argument order of mesh.cpp:13 */
};

struct alignas(16) TriExtension {
    alignas(16) Float3 n0;
    alignas(16) Float3 n1;
    alignas(16) Float3 n2;
    alignas(8) Float2 uv0;
    alignas(8) Float2 uv1;
    alignas(8) Float2 uv2;
};

class Mesh {
public:
    explicit Mesh(const std::string& path);      /* reads .obj or .obj.gz; throws std::runtime_error */
    Mesh(const std::string& path, unsigned threads);   /* parallel parse; same arrays for any thread count */
    Mesh() = default;
    std::vector<Triangle> triangles;
    std::vector<TriExtension> triExtensions;
};

/* ------------------------------------------------------------ BVH */
struct alignas(16) AABB {
    alignas(16) Float3 bbMin = Float3(INFINITY);
    alignas(16) Float3 bbMax = Float3(-INFINITY);
    void grow(const Float3& p) { bbMin = min(bbMin, p); bbMax = max(bbMax, p); }
    void grow(const AABB& b) { bbMin = min(bbMin, b.bbMin); bbMax = max(bbMax, b.bbMax); }
    F32 area() const;
    Float3 center() const;                        /* the reference's half-extent quirk, bvh.cpp:35-38 */
};

struct alignas(16) BvhNode {
    U32 leftFirst;
    U32 count;
    AABB boundingBox;
    bool isLeaf() const { return count != 0; }
};

/* Threads of the parallel BVH build: SURF_BUILD_THREADS, else OMP_NUM_THREADS,
 * else the hardware concurrency (capped at 64). */
unsigned defaultBuildThreads();

class BvhBLAS {
public:
    explicit BvhBLAS(Mesh* mesh);
    BvhBLAS(Mesh* mesh, unsigned threads);
    void build();                                 /* SURF_BUILD_THREADS / OMP_NUM_THREADS threads */
    void build(unsigned threads);                 /* same arrays for every thread count */
    void refit();
    const Mesh* mesh() const { return m_mesh; }
    SizeType triCount() const { return m_mesh->triangles.size(); }
    const U32* indices() const { return m_indices.data(); }
    U32 nodesUsed() const { return m_nodesUsed; }
    const BvhNode* nodePool() const { return m_nodes.data(); }
    const AABB& bounds() const { return m_nodes[0].boundingBox; }
    U32 depth() const;
private:
    Mesh* m_mesh;
    std::vector<U32> m_indices;
    std::vector<BvhNode> m_nodes;
    U32 m_nodesUsed = 2;
};

struct Material {
    alignas(4) F32 emissionStrength = 0.0f;
    alignas(4) F32 reflectivity = 0.0f;
    alignas(4) F32 refractivity = 0.0f;
    alignas(4) F32 indexOfRefraction = 1.0f;
    alignas(16) Float3 emissionColor = Float3(0.0f);
    alignas(16) Float3 albedo = Float3(0.0f);
    alignas(16) Float3 absorption = Float3(0.0f);
    bool isLight() const { return emissionStrength > 0.0f && (emissionColor.x > 0.0f || emissionColor.y > 0.0f || emissionColor.z > 0.0f); }
};

using GPUInstance = surf_gpu_instance;

class Instance {
public:
    Instance(BvhBLAS* blas, Material* material, Mat4 transform);
    const Mat4& transform() const { return m_transform; }
    void setTransform(const Mat4& transform);
    GPUInstance toGPUInstance() const;
    void updateInstanceData() { updateBounds(); }
    BvhBLAS* bvh;
    Material* material;
    AABB bounds;
    F32 area = 0.0f;
private:
    void updateBounds();
    void calculateMeshArea();
    Mat4 m_transform;
    Mat4 m_invTransform;
};

class BvhTLAS {
public:
    explicit BvhTLAS(std::vector<Instance> instances);
    void build();
    void refit();
    Instance& instance(SizeType i) { return m_instances[i]; }
    const std::vector<Instance>& instances() const { return m_instances; }
    const U32* indices() const { return m_indices.data(); }
    U32 nodesUsed() const { return m_nodesUsed; }
    const BvhNode* nodePool() const { return m_nodes.data(); }
    U32 depth() const;
private:
    std::vector<Instance> m_instances;
    std::vector<U32> m_indices;
    std::vector<BvhNode> m_nodes;
    U32 m_nodesUsed = 2;
};

/* ------------------------------------------------------------ scene */
enum class BackgroundType : U32 { SolidColor = 0, ColorGradient = 1 };

struct SceneBackground {
    alignas(4) BackgroundType type = BackgroundType::SolidColor;
    alignas(16) Float3 color = Float3(0.0f);
    struct {
        alignas(16) Float3 colorA = Float3(0.0f);
        alignas(16) Float3 colorB = Float3(0.0f);
    } gradient;
};

struct GPULightData { U32 lightInstanceIdx; U32 primitiveCount; };

struct GPUBatchInfo {
    std::vector<Triangle> triBuffer;
    std::vector<TriExtension> triExtBuffer;
    std::vector<U32> BLASIndices;
    std::vector<BvhNode> BLASNodes;
    std::vector<Material> materials;
    std::vector<GPUInstance> gpuInstances;
    std::vector<GPULightData> lights;
};

class GPUBatcher {
public:
    /* First-use order for meshes, BLASes and materials (the reference keys them
     * by pointer, an address-dependent but equivalent order). */
    static GPUBatchInfo createBatchInfo(const std::vector<Instance>& instances);
};

/* HIP device handle standing in for the reference's Vulkan RenderContext. */
struct RenderContext {
    int hipDevice = 0;
};

class GPUScene {
public:
    GPUScene(RenderContext* context, SceneBackground background, std::vector<Instance> instances);
    const SceneBackground& backgroundSettings() const { return m_background; }
    /* Scene::update / GPUScene::update (scene.cpp:267-282): rotate instance 3, refit, re-batch. */
    void update(F32 deltaTime);
    /* The scene as the C-ABI takes it (pointers into this object). */
    surf_scene_desc descriptor() const;
    const BvhTLAS& tlas() const { return m_sceneTlas; }
    U32 generation() const { return m_generation; }
    RenderContext* context() const { return m_context; }
private:
    RenderContext* m_context;
    SceneBackground m_background;
    BvhTLAS m_sceneTlas;
    GPUBatchInfo m_batchInfo;
    U32 m_generation = 0;
};

/* ------------------------------------------------------------ camera */
using CameraUBO = surf_camera_ubo;

struct ViewPlane { Float3 firstPixel, uVector, vVector; };

class Camera {
public:
    Camera(Float3 position, Float3 target, U32 screenWidth, U32 screenHeight, F32 fovY,
           F32 focalLength = 1.5f, F32 defocusAngle = 0.0f);
    Float3 right() const { return up.cross(forward).normalize(); }
    void generateViewPlane();
    CameraUBO toUBO() const;                      /* renderer.cpp:972-979 */
    Float3 position, forward, up;
    F32 screenWidth, screenHeight, fovY, focalLength, defocusAngle;
    ViewPlane viewPlane;
};

/* ------------------------------------------------------------ renderer */
struct RendererConfig {
    U32 maxBounces = 5;          /* unused by the reference's iterative path; kept */
    U32 samplesPerFrame = 1;     /* > 1: the throughput cutoff is off (surf_set_zero_cutoff's automatic default), so a
                                    lens TIR orbit runs to its end as in the reference -- up to millions of segments
                                    (seconds) for the frame holding it; maxSegments bounds it (surf_hip.h) */
    U32 maxSegments = 0;         /* 0: unbounded + Russian roulette (reference); N: cap (config C2) */
    bool lumenOutput = false;    /* WF_LUMEN_OUTPUT (renderer.cpp:31, default 0): frameInfo().energy from the
                                    accumulator; reading it drains the sample stream, so it is computed only
                                    when frameInfo() is read after a render */
};

struct FrameInstrumentationData {
    F32 energy = 0.0f;
    U32 totalSamples = 0;
};

struct FramebufferSize { U32 width, height; };

class UIManager;   /* accepted for signature compatibility, never used */

class IRenderer {
public:
    virtual ~IRenderer() = default;
    virtual void clearAccumulator() = 0;
    virtual void render(F32 deltaTime) = 0;
    virtual RendererConfig& config() = 0;
    virtual const FrameInstrumentationData& frameInfo() = 0;
};

class WaveFrontRenderer : public IRenderer {
public:
    WaveFrontRenderer(RenderContext* context, UIManager* uiManager, RendererConfig config,
                      FramebufferSize resolution, Camera& camera, GPUScene& scene);
    ~WaveFrontRenderer() override;
    WaveFrontRenderer(const WaveFrontRenderer&) = delete;
    WaveFrontRenderer& operator=(const WaveFrontRenderer&) = delete;

    void clearAccumulator() override;
    void render(F32 deltaTime) override;
    RendererConfig& config() override { return m_config; }
    const FrameInstrumentationData& frameInfo() override;

    /* headless additions */
    std::vector<F32> readAccumulator();           /* width*height*4 floats */
    std::vector<U32> finalizeRGBA8();             /* width*height RGBA8 words */
    std::vector<U32> displayRGBA8();              /* finalize image through fs_quad.frag's sqrt gamma */
    void synchronize();                           /* waits until every frame rendered so far is accumulated */
    surf_ctx* handle() const { return m_ctx; }
private:
    surf_ctx* m_ctx = nullptr;
    RendererConfig m_config;
    FramebufferSize m_resolution;
    Camera& m_camera;
    GPUScene& m_scene;
    U32 m_sceneGeneration = 0;
    U32 m_totalSamples = 0;
    FrameInstrumentationData m_frameInfo;
    bool m_energyStale = false;
};

static_assert(sizeof(Triangle) == sizeof(surf_triangle), "Triangle layout");
static_assert(sizeof(TriExtension) == sizeof(surf_tri_extension), "TriExtension layout");
static_assert(sizeof(BvhNode) == sizeof(surf_bvh_node), "BvhNode layout");
static_assert(sizeof(Material) == sizeof(surf_material), "Material layout");
static_assert(sizeof(SceneBackground) == sizeof(surf_background), "SceneBackground layout");
static_assert(sizeof(GPULightData) == sizeof(surf_light), "GPULightData layout");

}  // namespace surf
