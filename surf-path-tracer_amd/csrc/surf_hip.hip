/*
 * surf_hip.hip -- C-ABI implementation (include/surf_hip.h): device context,
 * scene upload + re-layout, the wavefront render loop (hipGraph-captured
 * phases), readback.  Replaces WaveFrontRenderer's Vulkan orchestration
 * (renderer.cpp:604-1454) -- without its per-bounce host round trip: the
 * host only polls a pinned counter block once per replayed graph of
 * kPhasesPerGraph phases.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cfloat>
#include <array>
#include <map>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

#include "surf_hip.h"
#include "device/wavefront_kernels.h"

using namespace surfdev;

namespace {

/* phases per full replay: 16 (C3 515.2 / 513.9 → 520.7 / 520.0 Mrays/s against
 * 8 on one box, C4, the drop-in loop and the 8-shard projection unchanged;
 * MEASUREMENTS r6) */
#ifndef SURF_PHASES_GRAPH
#define SURF_PHASES_GRAPH 16
#endif
constexpr int kPhasesPerGraph = SURF_PHASES_GRAPH;   /* even: parity returns to 0 after a replay */
static_assert(kPhasesPerGraph % 2 == 0, "even: parity returns to 0 after a replay");
/* The short graph: a render call with at most one frame left to issue (the
 * drop-in loop's 1-spp render(), main.cpp:381-446) replays 4 phases per host
 * poll instead of 8, so a per-frame call does not keep the pool a quarter full
 * for 8 phases per frame.  4096 one-frame calls at 1280x720: 625 / 641 / 637
 * Mrays/s with 2 / 4 / 8 phases (each replay's end joins its last k_connect,
 * which then overlaps nothing; MEASUREMENTS round 5). */
#ifndef SURF_PHASES_SHORT
#define SURF_PHASES_SHORT 4
#endif
constexpr int kPhasesShort = SURF_PHASES_SHORT;
static_assert(kPhasesShort % 2 == 0 && kPhasesShort <= kPhasesPerGraph, "even: parity returns to 0 after a replay");
constexpr int kPhaseEvents = 6;             /* profiling events per phase: sort, extend, shade, sort, connect, regen */
constexpr uint32_t kMaxStack = 120;          /* LDS stack entries per ray (block 256 -> 120 KiB max) */
constexpr uint64_t kMaxIterations = 1ull << 22;  /* safety net: a path longer than this is a bug */

std::mutex gErrMutex;
std::string gLastError;

void setGlobalError(const std::string& e) { std::lock_guard<std::mutex> l(gErrMutex); gLastError = e; }

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

}  // namespace

struct surf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t width = 0, height = 0;
    std::vector<uint32_t> rows;
    uint32_t npx = 0;
    uint32_t capacity = 0;
    uint32_t window = 0;           /* frames whose samples may be in flight (radiance slots; ensureWindow) */
    bool windowFixed = false;      /* set by surf_set_frame_batch */
    bool profiling = false;
    std::string err;

    /* scene */
    bool hasScene = false;
    uint32_t extBlock = 128;       /* k_extend workgroup size (SURF_EXTEND_BLOCK=128|256): 128 measured 5 % faster on k_extend */
    bool connectGlobal = false;    /* k_connect reads its tables from global memory (SURF_CONNECT_GLOBAL=1, tuning) */
    bool extStack16 = true;        /* k_extend's stack in 16-bit entries when node indices fit (SURF_EXT_STACK16=0: 32-bit) */
    bool regenCount = true;        /* k_regen_count fills the next pool and counts it for its sort (SURF_REGEN_COUNT=0: k_regen + k_bincount) */
    /* the lane walk leaves a ray after laneCap node visits of one BLAS walk
     * to k_extend_cont (SURF_LANE_CAP; 0 = off, the default: measured slower) */
    uint32_t laneCap = 0;
    uint32_t* resumeRec = nullptr;  /* resume records, 64 words each (allocated with the first capped graph) */
    uint32_t resumeCap = 0;
    bool ldsTables = false;        /* instance/material/light tables fit the per-workgroup LDS copy */
    DevScene S{};
    std::vector<void*> sceneAllocs;
    uint32_t stackDepth = 0;
    uint32_t nInstances = 0, nTriangles = 0, nBlasNodes = 0;
    /* what surf_update_instances may change: instance records, TLAS, lights */
    uint32_t nMaterials = 0, nLightsUp = 0, tlasNodeCount = 0, maxBlasDepth = 0;
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, std::array<float4, 4>> blasRoots;  /* (node, idx, tri offset) -> root record */
    std::map<uint32_t, std::array<double, 6>> blasBounds;   /* tri offset -> bounds of its BLAS's triangles (v0, v0+e1, v0+e2) */
    std::map<uint32_t, uint32_t> blasSlots;                  /* tri offset -> index slots (triangles) of its BLAS */
    /* issue order: the pixels whose centre ray first hits a heavy instance
     * (long Russian-roulette paths start there) are issued for all frames of a
     * multi-frame stream before the rest (SURF_REORDER=0: frame-major) */
    bool reorder = true;
    bool permValid = false;
    uint32_t* dPerm = nullptr;
    /* one-frame render calls may leave up to a pool of their stream unissued
     * (SURF_LOOP_LAG=0: issue each call's frame before returning) */
    bool loopLag = true;
    /* occupancy probes: extra dynamic LDS per k_extend / k_connect workgroup (SURF_EXT_LDS_PAD / SURF_CON_LDS_PAD bytes) */
    size_t extLdsPad = 0, conLdsPad = 0;
    /* k_connect stages the emitters' BLAS node records in LDS when they are
     * few and every BLAS node index fits 16 bits (SURF_LDS_LIGHTBLAS=0: never) */
    bool ldsLightBlas = true;
    /* small BLASes in the compact form k_connect stages (blasAnyStaged): BLAS
     * node offset -> interior records on the device, their count, index offset, triangle slots */
    struct StagedBlas { const float4* rec; uint32_t recN, tri0, triN; };
    std::map<uint32_t, StagedBlas> stagedBlas;
    uint32_t permA = 0, permFrames = 0;
    std::vector<uint32_t> heavyInst;
    /* pool ray-order key (SURF_KEY): 2 heavy-instance mask x quadrant, most
     * heavy instances first (the default: the costliest rays are dealt to the
     * first-dispatched workgroups, DESIGN 4 "Pool sizing"), 1 the same key
     * ascending, 0 start instance x quadrant */
    uint32_t keyMode = 2;
    /* camera */
    bool hasCamera = false;
    DevCamera cam{};
    surf_camera_ubo camUbo{};

    /* wavefront state */
    bool allocated = false;
    Pool pool[2]{};
    float4* hitTUV = nullptr;
    uint32_t* hitInst = nullptr;
    ShadowQ Q{};
    float4* rad = nullptr;
    float4* acc = nullptr;
    uint32_t* dRows = nullptr;
    Counters* ctr = nullptr;
    Counters* hctr = nullptr;      /* pinned: the counters as of the last consumed snapshot */
    uint32_t* frameDone = nullptr; /* [kStripes][window] completions per frame slot */
    /* host snapshots of the counters and of the open passes' completion
     * stripes, each taken after a graph replay; a lagged one-frame call may
     * return with up to kSnaps of them (and their replays) in flight, so the
     * GPU keeps working while the application runs its loop (pump) */
    struct Snap { Counters* h = nullptr; uint32_t* fd = nullptr; uint64_t acc = 0, open = 0; int phases = 0; hipEvent_t ev = nullptr; };
    static constexpr int kSnaps = 2;
    Snap snap[kSnaps];
    int snapHead = 0, snapCount = 0;
    uint64_t issuePerPhase = 0;    /* chains a phase issued in the last unstarved snapshot of this stream: what the replays in flight will issue */
    bool pipeline = true;          /* SURF_PIPELINE=0: every replay waited for before the next (and before a call returns) */
    /* issue limits pushed to the device: a ring of pinned sources, so a later
     * push never rewrites the bytes an earlier, still queued copy reads */
    static constexpr uint32_t kLimitRing = 16;
    uint64_t* hLimit = nullptr;
    uint32_t hLimitNext = 0;
    /* device time of calls that return with replays in flight: two event
     * pairs used in turn, read once their end has passed */
    hipEvent_t tev[2][2] = {};
    bool tevPending[2] = {false, false};
    int tevCur = 0;
    uint32_t* dOutRGBA = nullptr;
    std::vector<void*> wfAllocs;
    uint64_t totalSamples = 0;     /* frames rendered since the last clear (samples per pixel) */

    /* sample stream: targetFrames frames of spp samples per pixel requested,
     * i.e. passes (samples per pixel) [0, targetFrames * spp) after the
     * baseFrame samples rendered before the stream; pass q lives in radiance
     * slot q % window (window a multiple of spp) */
    bool streamActive = false;
    uint64_t baseFrame = 0;        /* sample count before the stream (the reference's totalSamples) */
    uint64_t targetFrames = 0;     /* frames requested (chains per pixel) */
    uint64_t accPasses = 0;        /* passes accumulated (in order) */
    uint32_t spp = 1;              /* samples per frame of the stream (a frame's samples chain their RNG state) */
    uint32_t streamMaxSeg = 0;
    int zeroCutoff = -1;           /* early end of paths with throughput < FLT_MIN: 1 on, 0 off, -1 automatic (on for 1-sample frames) */
    uint64_t pushedLimit = 0;
    uint32_t tailPaths = 0;        /* drain policy (surf_set_tail_policy), 0 = automatic */
    uint32_t tailBudget = 16;      /* per-stage segment budget of the drain tail (0 = one stage); 16: measured fastest */
    Pool surv[2]{};                /* drain survivors, ping-pong between stages */
    uint32_t survCap = 0;
    uint32_t coopMax = 0;          /* survivors handled by the cooperative tail (one path per wave) */
    uint32_t coopAll = 150000;     /* drain paths left to the cooperative tail (surf_set_tail_coop); C3 drain 176-184 ms at 60000, 172-178 at 150000 */
    int drainReplays = 1;          /* graph replays per host poll while draining (SURF_DRAIN_REPLAYS) */
    bool drainShort = false;       /* short replays once nothing is left to issue (SURF_DRAIN_SHORT=1; measured slower, MEASUREMENTS round 5) */
    bool regenFirst = false;       /* k_regen before the connect fork (SURF_REGEN_FIRST=1; measured equal, MEASUREMENTS round 5) */
    int traceMode = 0;             /* surf_trace_closest/_any: 0 one ray per lane, 1 one ray per wave */
    bool connectStaged = false;    /* the last k_connect launched walked the emitters' BLAS from LDS (surf_debug_connect_staging) */
    bool tailPair = true;          /* cooperative drain on k_tail_pair (partner waves trace the shadow rays; SURF_TAIL_PAIR=0: k_tail_coop) */
    uint32_t cus = 256;            /* compute units of the device */
    bool sortRays = true;          /* order each phase's rays by start instance (SURF_SORT=0: off) */
    bool sortPool = true;
    bool sortShadow = true;        /* ... and the shadow queue by light (SURF_SORT=2: pool only, 3: shadow queue only) */
    /* ray order: counts from k_regen_count (or k_bincount), then k_binscatter each phase */
    uint32_t* order = nullptr;
    uint32_t* binHist = nullptr;
    /* connect overlapped with the next phase's regen / pool sort / extend
     * (SURF_OVERLAP=0: one stream): its own stream in the graph capture, its
     * own shadow order and histograms */
    bool overlap = true;
    hipStream_t side = nullptr;
    hipEvent_t capEv[2 * kPhasesPerGraph] = {};
    uint32_t tailLanes = 0;
    uint32_t segMaxBase = 0;       /* longest path of finished streams */
    uint64_t tailFirstRays = 0;    /* first extension rays of drained paths: counted by regen, traced by the tail */

    /* graph */
    hipGraphExec_t graphExec = nullptr, graphExecShort = nullptr;
    hipGraph_t graph = nullptr, graphShort = nullptr;
    uint32_t gridWork = 0, gridRegen = 0, gridExtend = 0, gridConnect = 0;

    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t pev[kPhasesPerGraph * kPhaseEvents + 1] = {};   /* profiling: kPhaseEvents per phase + the end */
    uint32_t* hPhaseN = nullptr;   /* profiling + SURF_PHASE_LOG: paths each phase extends (pinned) */
    FILE* phaseLog = nullptr;      /* SURF_PHASE_LOG=<file>: one line per profiled phase (size, kernel ms) */
    surf_stats stats{};
    unsigned long long evBase[kEvents] = {};   /* event counts of finished streams since the last clear */
};

#define SURF_CHECK(ctx, call)                                                             \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess) {                                                           \
            (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e_);               \
            setGlobalError((ctx)->err);                                                   \
            return SURF_ERR_HIP;                                                          \
        }                                                                                 \
    } while (0)

namespace {

int fail(surf_ctx* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    setGlobalError(msg);
    return code;
}

template <class T>
int devAlloc(surf_ctx* c, std::vector<void*>& list, T** out, size_t count) {
    *out = nullptr;
    if (count == 0) count = 1;
    void* p = nullptr;
    if (hipMalloc(&p, count * sizeof(T)) != hipSuccess || !p) {
        return fail(c, SURF_ERR_OOM, "hipMalloc of " + std::to_string(count * sizeof(T)) + " bytes failed");
    }
    list.push_back(p);
    *out = static_cast<T*>(p);
    return SURF_OK;
}

void freeList(std::vector<void*>& list) {
    for (void* p : list) (void)hipFree(p);
    list.clear();
}

void destroyGraph(surf_ctx* c) {
    if (c->graphExec) (void)hipGraphExecDestroy(c->graphExec);
    if (c->graph) (void)hipGraphDestroy(c->graph);
    if (c->graphExecShort) (void)hipGraphExecDestroy(c->graphExecShort);
    if (c->graphShort) (void)hipGraphDestroy(c->graphShort);
    c->graphExec = c->graphExecShort = nullptr;
    c->graph = c->graphShort = nullptr;
}

/* Dynamic LDS of a traversal kernel with `block` threads: the per-lane stack,
 * then (LDS tables) the TraceInst table and the TLAS index array. */
uint32_t stackWords(const surf_ctx* c, uint32_t block) { return c->stackDepth * block; }
/* one-ray-per-wave traversal (traceWave): a stack of node records, 16 words per
 * entry -- 64 with two-level records (blasWalk2 pushes whole W records) */
uint32_t recStackWords(const surf_ctx* c) { return c->stackDepth * (c->S.wnodes ? 64u : 16u); }
/* Dynamic LDS of the one-ray-per-wave kernels: the record stack, the prologue
 * table (16 words per instance), then the trace tables; k_tail_coop adds the
 * shading tables (coopTailLds). */
/* (tables staged only when they fit: coopLdsTables in the kernels) */
size_t coopLds(const surf_ctx* c) {
    return ((size_t)recStackWords(c) + 16u * c->nInstances) * sizeof(float) +
           (c->ldsTables ? (size_t)c->nInstances * (sizeof(TraceInst) + sizeof(uint32_t)) : 0);
}
size_t coopTailLds(const surf_ctx* c) {
    if (!c->ldsTables) return coopLds(c);
    return ((coopLds(c) + 15) & ~(size_t)15) + (size_t)c->nInstances * sizeof(DevInstance) + (size_t)c->nMaterials * sizeof(DevMaterial) +
           (size_t)c->nLightsUp * sizeof(uint2);
}
/* k_tail_pair: a record stack and a prologue table per wave (two waves), then the tables */
size_t pairTailLds(const surf_ctx* c) {
    return coopTailLds(c) + ((size_t)recStackWords(c) + 16u * c->nInstances) * sizeof(float);
}
/* the one-ray-per-wave kernels' LDS: stack + prologue table per wave (+ tables) within 64 KiB */
bool coopLdsOk(const surf_ctx* c) { return pairTailLds(c) <= 65536; }
size_t traversalLds(const surf_ctx* c, uint32_t block) {
    size_t b = (size_t)stackWords(c, block) * sizeof(uint32_t);
    if (c->ldsTables) b += (size_t)c->nInstances * (sizeof(TraceInst) + sizeof(uint32_t));
    return b;
}

/* ----------------------------------------------------------- scene upload
 * Walks every BLAS/TLAS from its root: validates indices (no kernel can
 * fault on a malformed scene), measures depth, and emits the device node
 * record that carries the children's boxes. */
struct TreeWalk {
    uint32_t depth = 0;
    bool ok = true;
    std::string why;
};

TreeWalk walkTree(const surf_bvh_node* nodes, uint32_t nodeCount, uint32_t offset, uint32_t idxCount, uint32_t idxOffset,
                  std::vector<float4>& out, std::vector<uint8_t>& leafSeen, std::vector<uint32_t>* owner = nullptr) {
    TreeWalk w;
    std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 0u}};
    size_t visits = 0;
    while (!st.empty()) {
        auto [local, dep] = st.back();
        st.pop_back();
        if (++visits > (size_t)nodeCount + 1 || dep > 4096) { w.ok = false; w.why = "BVH has a cycle"; return w; }
        const uint64_t g = (uint64_t)offset + local;
        if (g >= nodeCount) { w.ok = false; w.why = "BVH node index out of range"; return w; }
        const surf_bvh_node& n = nodes[g];
        float4* rec = &out[4 * g];
        if (owner) (*owner)[g] = offset;
        rec[0].w = u2f(n.left_first);
        rec[1].w = u2f(n.count);
        if (n.count != 0) {
            if ((uint64_t)idxOffset + n.left_first + n.count > idxCount) { w.ok = false; w.why = "BVH leaf range out of range"; return w; }
            for (uint32_t k = 0; k < n.count; ++k) leafSeen[idxOffset + n.left_first + k] = 1;
            w.depth = std::max(w.depth, dep);
            continue;
        }
        const uint64_t l = (uint64_t)offset + n.left_first;
        if (l + 1 >= nodeCount) { w.ok = false; w.why = "BVH child index out of range"; return w; }
        const surf_bvh_node& L = nodes[l];
        const surf_bvh_node& R = nodes[l + 1];
        rec[0] = make_float4(L.bb_min.x, L.bb_min.y, L.bb_min.z, rec[0].w);
        rec[1] = make_float4(L.bb_max.x, L.bb_max.y, L.bb_max.z, rec[1].w);
        rec[2] = make_float4(R.bb_min.x, R.bb_min.y, R.bb_min.z, 0.0f);
        rec[3] = make_float4(R.bb_max.x, R.bb_max.y, R.bb_max.z, 0.0f);
        st.push_back({n.left_first + 1, dep + 1});
        st.push_back({n.left_first, dep + 1});
    }
    return w;
}

template <class T>
int upload(surf_ctx* c, const std::vector<T>& host, const T** devOut) {
    T* d = nullptr;
    int rc = devAlloc(c, c->sceneAllocs, &d, host.size());
    if (rc) return rc;
    if (!host.empty()) SURF_CHECK(c, hipMemcpy(d, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice));
    *devOut = d;
    return SURF_OK;
}

int allocWavefront(surf_ctx* c) {
    if (c->allocated) return SURF_OK;
    if (c->capacity == 0) {
        /* default: 5 full frames of paths in flight, bounded at 16M paths
         * (measured, DESIGN §4 "Pool sizing": C3 435-439 -> 470-475 Mrays/s
         * from 4 to 5 frames, 4.5 frames no better than 4, 6 slower again).
         * Sized from the whole frame, not the shard: a row shard of G GPUs
         * keeps the same pool, so its stream needs ~G times fewer wavefront
         * phases (each phase pays launch and poll latency however few paths it
         * holds). */
        const uint64_t want = (uint64_t)c->width * c->height * 5;
        c->capacity = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(want, 65536), 1u << 24);
    }
    const size_t cap = c->capacity;
    int rc;
    for (int p = 0; p < 2; ++p) {
        if ((rc = devAlloc(c, c->wfAllocs, &c->pool[p].od, 2 * cap))) return rc;
        if ((rc = devAlloc(c, c->wfAllocs, &c->pool[p].T, cap))) return rc;
        if ((rc = devAlloc(c, c->wfAllocs, &c->pool[p].key, cap))) return rc;
    }
    if ((rc = devAlloc(c, c->wfAllocs, &c->order, cap))) return rc;
    if ((rc = devAlloc(c, c->wfAllocs, &c->binHist, (size_t)kBins * kSortBlocks))) return rc;
    if ((rc = devAlloc(c, c->wfAllocs, &c->dPerm, c->npx))) return rc;
    /* grid: 8 workgroups of 256 per CU saturate the 256-CU chip; grid-stride beyond */
    int cus = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c->device) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
    /* drain stages: survivors of a tail stage, ping-pong */
    c->survCap = (uint32_t)std::min<size_t>(std::max<size_t>(cap / 16, 4096), 1u << 18);
    for (int q = 0; q < 2; ++q) {
        if ((rc = devAlloc(c, c->wfAllocs, &c->surv[q].od, 2 * (size_t)c->survCap))) return rc;
        if ((rc = devAlloc(c, c->wfAllocs, &c->surv[q].T, c->survCap))) return rc;
    }
    if ((rc = devAlloc(c, c->wfAllocs, &c->hitTUV, cap))) return rc;
    if ((rc = devAlloc(c, c->wfAllocs, &c->hitInst, cap))) return rc;
    /* shadow queue: kShBins bin regions of a quarter pool each (a phase queues
     * at most one shadow ray per path; C3 puts <= 30 % of them in one bin), then
     * an overflow region of a whole pool */
    c->Q.region = (uint32_t)((cap / (4 * kShXcds) + 255) / 256 * 256);
    c->Q.bins = (c->sortRays && c->sortShadow) ? kShBins : 1u;
    const size_t qslots = (size_t)(kShSegs - 1) * c->Q.region + cap;
    if ((rc = devAlloc(c, c->wfAllocs, &c->Q.od, 2 * qslots))) return rc;
    if ((rc = devAlloc(c, c->wfAllocs, &c->Q.c, qslots))) return rc;
    if ((rc = devAlloc(c, c->wfAllocs, &c->Q.cur, (size_t)2 * kShSegs * kShStride))) return rc;
    if ((rc = devAlloc(c, c->wfAllocs, &c->ctr, 1))) return rc;
    if ((rc = devAlloc(c, c->wfAllocs, &c->dOutRGBA, c->npx))) return rc;
    if (hipHostMalloc((void**)&c->hctr, sizeof(Counters), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&c->hLimit, surf_ctx::kLimitRing * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess)
        return fail(c, SURF_ERR_OOM, "hipHostMalloc of the counter block failed");
    for (auto& sn : c->snap) {
        if (hipHostMalloc((void**)&sn.h, sizeof(Counters), hipHostMallocDefault) != hipSuccess)
            return fail(c, SURF_ERR_OOM, "hipHostMalloc of a counter snapshot failed");
        SURF_CHECK(c, hipEventCreateWithFlags(&sn.ev, hipEventDisableTiming));
    }
    for (auto& pr : c->tev)
        for (auto& e : pr) SURF_CHECK(c, hipEventCreate(&e));
    for (auto& e : c->pev) SURF_CHECK(c, hipEventCreate(&e));
    if (const char* e = std::getenv("SURF_PHASE_LOG")) {         /* diagnostics: per-phase cost vs size */
        if (hipHostMalloc((void**)&c->hPhaseN, kPhasesPerGraph * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
            return fail(c, SURF_ERR_OOM, "hipHostMalloc of the phase log failed");
        c->phaseLog = std::fopen(e, "a");
    }
    const uint64_t maxBlocks = (cap + kBlock - 1) / kBlock;
    uint64_t perCu = 8;                                   /* workgroups per CU of the wavefront kernels (SURF_GRID_PER_CU) */
    if (const char* e = std::getenv("SURF_GRID_PER_CU")) perCu = (uint64_t)std::max(1, std::atoi(e));
    c->gridWork = (uint32_t)std::min<uint64_t>(maxBlocks, (uint64_t)cus * perCu);
    /* per-kernel grids (measured): k_extend gains from one ray per
     * thread (latency hiding across many short-lived blocks), k_connect peaks
     * at 14-15 workgroups per CU with its LDS-staged light BLAS (5 resident:
     * the dispatcher rebalances the grid-stride chunks; past ~15 every extra
     * workgroup re-stages the BLAS -- MEASUREMENTS round 5), k_shade at 8 */
    uint64_t extPerCu = 48, conPerCu = 15;
    const char* eExt = std::getenv("SURF_GRID_EXTEND");
    if (eExt) extPerCu = (uint64_t)std::max(1, std::atoi(eExt));
    if (const char* e = std::getenv("SURF_GRID_CONNECT")) conPerCu = (uint64_t)std::max(1, std::atoi(e));
    if (c->extBlock == 128) extPerCu *= 2;                 /* the same threads per CU in half-size workgroups */
    c->gridExtend = (uint32_t)std::min<uint64_t>((cap + c->extBlock - 1) / c->extBlock, (uint64_t)cus * extPerCu);
    /* k_extend: ~1.5 rays per thread at a full pool (grid-stride).  Measured
     * (DESIGN §4 "Pool sizing"): with the heavy-first ray order the launch
     * time is flat from 1.2 to 1.5 rays per thread (C3 117-118 ms per render at
     * 48-56 workgroups per CU), slower at one ray per thread (131 ms) and at
     * >= 1.7 (C3 127 ms at 36; C4: 1.56 -> 1094 ms, 3.1 -> 1170 ms) */
    if (!eExt) c->gridExtend = (uint32_t)std::max<uint64_t>(c->gridExtend, (cap * 2 / 3 + c->extBlock - 1) / c->extBlock);
    c->gridConnect = (uint32_t)std::min<uint64_t>(maxBlocks, (uint64_t)cus * conPerCu);
    c->coopMax = (uint32_t)cus * 4 * SURF_TAIL_WAVES;
    c->cus = (uint32_t)cus;
    if (const char* e = std::getenv("SURF_DRAIN_REPLAYS")) c->drainReplays = std::max(1, std::atoi(e));
    c->gridRegen = (uint32_t)std::min<uint64_t>(maxBlocks, (uint64_t)cus * 8);
    c->allocated = true;
    return SURF_OK;
}

/* The radiance ring (float4 per frame slot x pixel) and the per-slot
 * completion counters, sized for the stream about to start (no stream active):
 * as many slots as the stream requests frames -- so no frame waits for an old
 * frame's long Russian-roulette paths to free a slot -- at least kWindowFloor,
 * and at least kLoopFloor for a stream opened by a one-frame request (a
 * drop-in loop extends its stream one frame per call, so its first request
 * says nothing about its length; 4096 one-frame calls at 1280x720 run at
 * 552 / 593 / 614 Mrays/s with 1024 / 2048 / 4096 slots, MEASUREMENTS round 5), at most
 * 4096 and at most what min(64 GiB, a quarter of the free HBM) holds (HBM3E:
 * 288 GB per GPU; 4096 slots at 1280x720 take 60 GB).  A
 * later, longer stream grows the ring; a window set by surf_set_frame_batch
 * is kept as given. */
constexpr uint64_t kWindowFloor = 256, kLoopFloor = 4096;
constexpr uint64_t kLdsLightBlas = 20480;     /* k_connect's staged emitter BLAS (compact records + triangles), bytes at most */
int ensureWindow(surf_ctx* c, uint64_t frames, uint32_t spp) {
    const uint64_t passes = frames * spp;
    const uint64_t floor = frames == 1 ? kLoopFloor : kWindowFloor;
    uint64_t want = c->windowFixed ? c->window : std::min<uint64_t>(4096, std::max<uint64_t>(passes, floor));
    if (c->windowFixed && c->window % spp != 0)
        return fail(c, SURF_ERR_INVALID, "frame window " + std::to_string(c->window) + " is not a multiple of samples_per_frame " +
                                             std::to_string(spp));
    if (!c->windowFixed) {
        uint64_t budget = 64ull << 30;
        size_t freeB = 0, totalB = 0;
        if (hipMemGetInfo(&freeB, &totalB) == hipSuccess && freeB > 0)
            budget = std::min<uint64_t>(budget, (freeB + (c->rad ? (size_t)c->npx * c->window * sizeof(float4) : 0)) / 4);
        want = std::max<uint64_t>(1, std::min<uint64_t>(want, budget / ((uint64_t)c->npx * sizeof(float4))));
        /* a frame's samples take consecutive slots of one window turn */
        want = std::max<uint64_t>(spp, want / spp * spp);
        if ((uint64_t)c->npx * want >= (1ull << 32))
            return fail(c, SURF_ERR_OOM, "radiance ring of " + std::to_string(want) + " passes exceeds 32-bit sample ids");
        if (c->rad && want <= c->window && c->window % spp == 0) return SURF_OK;
    }
    if (c->rad && want == c->window) return SURF_OK;
    if (c->rad) {
        SURF_CHECK(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->rad); (void)hipFree(c->frameDone);
        for (auto& sn : c->snap) { (void)hipHostFree(sn.fd); sn.fd = nullptr; }
        c->rad = nullptr; c->frameDone = nullptr;
        destroyGraph(c);                          /* the ring and the window are kernel arguments */
    }
    c->window = (uint32_t)want;
    bool ok = hipMalloc(&c->rad, (size_t)c->npx * c->window * sizeof(float4)) == hipSuccess &&
              hipMalloc(&c->frameDone, (size_t)kStripes * c->window * sizeof(uint32_t)) == hipSuccess;
    for (auto& sn : c->snap)
        ok = ok && hipHostMalloc((void**)&sn.fd, (size_t)kStripes * c->window * sizeof(uint32_t), hipHostMallocDefault) == hipSuccess;
    if (!ok) {
        if (c->rad) (void)hipFree(c->rad);
        if (c->frameDone) (void)hipFree(c->frameDone);
        for (auto& sn : c->snap) { if (sn.fd) (void)hipHostFree(sn.fd); sn.fd = nullptr; }
        c->rad = nullptr; c->frameDone = nullptr;
        return fail(c, SURF_ERR_OOM, "radiance ring of " + std::to_string(c->window) + " frames does not fit");
    }
    return SURF_OK;
}

StreamGeom geom(const surf_ctx* c) { return StreamGeom{c->dRows, c->width, c->npx, c->window, c->dPerm}; }

/* The capped lane walk (LaneCap): a TLAS of one leaf of <= 64 instances and
 * a stack that fits a resume record */
bool laneCapOn(const surf_ctx* c) {
    return c->laneCap > 0u && c->S.tlasLeafCount >= 1u && c->S.tlasLeafCount <= 64u && c->stackDepth <= 64u - kResumeHead;
}

/* Counting sort of the pool (which 0) or shadow queue (which 1) of phase par
 * by its 4-bit key into c->order. */
void launchSort(surf_ctx* c, const uint8_t* key, int par, int which, hipStream_t st, uint32_t* hist, uint32_t* out, bool count = true) {
    if (count)   /* (else k_regen_count left the counts) */
        hipLaunchKernelGGL(k_bincount, dim3(kSortBlocks), dim3(kSortThreads), 0, st, key, (const Counters*)c->ctr, par, which, hist);
#if !SURF_SORT_FUSED_SCAN
    hipLaunchKernelGGL(k_binscan, dim3(1), dim3(1024), 0, st, hist, kBins * kSortBlocks);
#endif
    hipLaunchKernelGGL(k_binscatter, dim3(kSortBlocks), dim3(kSortThreads), 0, st, key, (const Counters*)c->ctr, par, which,
                       (const uint32_t*)hist, out);
}

/* One wavefront phase (ph = 0..kPhasesPerGraph-1): sort -> extend -> shade
 * -> sort -> connect -> regen.  With ev != null, ev[0..5] are recorded before
 * the pool sort, k_extend, k_shade, the shadow sort, k_connect and k_regen
 * (the phase ends at the next phase's ev[0]); everything on one stream.
 * Overlapped (graph capture, c->overlap): the shadow sort and k_connect of
 * phase ph run on the side stream, beside k_regen and the next phase's pool
 * sort and k_extend, which do not touch what they use (the shadow queue, its
 * order and histograms, the radiance of paths still being shaded); the next
 * k_shade waits for them: it reuses the shadow queue, and a path's NEE
 * contribution of bounce i must be added before what bounce i+1 adds. */
void launchPhase(surf_ctx* c, int ph, hipEvent_t* ev) {
    const int par = ph & 1;
    const uint32_t sw = stackWords(c, kBlock);
    const bool ovl = !ev && c->overlap;
    hipStream_t s0 = c->stream, s1 = ovl ? c->side : c->stream;
    if (ev && c->phaseLog)
        (void)hipMemcpyAsync(&c->hPhaseN[ph], &c->ctr->nIn[par], sizeof(uint32_t), hipMemcpyDeviceToHost, s0);
    if (ev) (void)hipEventRecord(ev[0], s0);
    const uint32_t* order = nullptr;
    const bool sortOn = c->sortRays && c->sortPool;
    const bool fused = sortOn && c->regenCount;    /* k_regen_count counts the next pool for its sort */
    if (sortOn) {
        launchSort(c, c->pool[par].key, par, 0, s0, c->binHist, c->order, !fused);
        order = c->order;
    }
    auto regen = [&]() {
        if (fused)
            hipLaunchKernelGGL(k_regen_count, dim3(kSortBlocks), dim3(kSortThreads), 0, s0, c->cam, c->pool[par ^ 1], c->rad, c->ctr,
                               par, c->capacity, geom(c), c->Q, c->binHist);
        else
            hipLaunchKernelGGL(k_regen, dim3(c->gridRegen), dim3(kBlock), 0, s0, c->cam, c->pool[par ^ 1], c->rad, c->ctr, par,
                               c->capacity, geom(c), c->Q);
    };
    if (ev) (void)hipEventRecord(ev[1], s0);
    const Pool cur = c->pool[par];                 /* the pool k_extend / k_shade read */
    /* LW: the two-level records in the lane traversal (HBM-resident BVHs, S.laneW) */
    /* 16-bit stack entries when every node index fits (the lane walk over
     * two-level records stacks 32-bit packed leaf references) */
    const bool sk16 = c->extStack16 && !c->S.laneW && c->nBlasNodes < 65536u && c->tlasNodeCount < 65536u;
    const bool capW = laneCapOn(c);
    auto extendK = c->S.laneW ? (capW ? (c->ldsTables ? k_extend<true, true, uint32_t, true> : k_extend<false, true, uint32_t, true>)
                                      : (c->ldsTables ? k_extend<true, true> : k_extend<false, true>))
                   : capW ? (sk16 ? (c->ldsTables ? k_extend<true, false, uint16_t, true> : k_extend<false, false, uint16_t, true>)
                                  : (c->ldsTables ? k_extend<true, false, uint32_t, true> : k_extend<false, false, uint32_t, true>))
                          : sk16 ? (c->ldsTables ? k_extend<true, false, uint16_t> : k_extend<false, false, uint16_t>)
                                 : (c->ldsTables ? k_extend<true, false> : k_extend<false, false>);
    const size_t extLds = traversalLds(c, c->extBlock) - (sk16 ? (size_t)stackWords(c, c->extBlock) * 2u : 0u);
    hipLaunchKernelGGL(extendK, dim3(c->gridExtend), dim3(c->extBlock), extLds + c->extLdsPad, s0, c->S,
                       cur, c->hitTUV, c->hitInst, (const Counters*)c->ctr, par, stackWords(c, c->extBlock), order,
                       c->laneCap, c->resumeRec, c->resumeCap);
    if (capW) {   /* the rays the capped lane walk left, 64 to a wave again (LaneCap) */
        auto contK = c->S.laneW ? (c->ldsTables ? k_extend_cont<true, true, uint32_t> : k_extend_cont<false, true, uint32_t>)
                     : sk16 ? (c->ldsTables ? k_extend_cont<true, false, uint16_t> : k_extend_cont<false, false, uint16_t>)
                            : (c->ldsTables ? k_extend_cont<true, false, uint32_t> : k_extend_cont<false, false, uint32_t>);
        hipLaunchKernelGGL(contK, dim3(std::min<uint32_t>((c->resumeCap + kBlock - 1) / kBlock, c->cus * 8u)), dim3(kBlock),
                           traversalLds(c, kBlock) - (sk16 ? (size_t)stackWords(c, kBlock) * 2u : 0u), s0, c->S, cur, c->hitTUV,
                           c->hitInst, (const Counters*)c->ctr, par, stackWords(c, kBlock), (const uint32_t*)c->resumeRec,
                           c->resumeCap);
    }
    if (ev) (void)hipEventRecord(ev[2], s0);
    if (ovl && ph > 0) (void)hipStreamWaitEvent(s0, c->capEv[2 * (ph - 1) + 1], 0);   /* the previous phase's connect */
    if (c->ldsTables)
        hipLaunchKernelGGL(k_shade<true>, dim3(c->gridWork), dim3(kBlock), 0, s0, c->S, cur, c->pool[par ^ 1],
                           c->hitTUV, (const uint32_t*)c->hitInst, c->Q, c->rad, c->frameDone, c->npx, c->window, c->ctr, par, order,
                           c->cam, geom(c));
    else
        hipLaunchKernelGGL(k_shade<false>, dim3(c->gridWork), dim3(kBlock), 0, s0, c->S, cur, c->pool[par ^ 1],
                           c->hitTUV, (const uint32_t*)c->hitInst, c->Q, c->rad, c->frameDone, c->npx, c->window, c->ctr, par, order,
                           c->cam, geom(c));
    if (ev) (void)hipEventRecord(ev[3], s0);
    /* k_regen before the fork (SURF_REGEN_FIRST): alone it takes ~17 us, beside
     * k_connect it waits for CU slots on the next phase's critical path */
    if (c->regenFirst) regen();
    if (ovl) {
        (void)hipEventRecord(c->capEv[2 * ph], s0);
        (void)hipStreamWaitEvent(s1, c->capEv[2 * ph], 0);
    }
    /* (the shadow rays are already in bin order: k_shade appends each to its
     * bin's region of the queue -- no sort pass) */
    if (ev) (void)hipEventRecord(ev[4], s0);
    const bool ldsC = c->ldsTables && !c->connectGlobal;   /* else global tables: LDS holds only the traversal stack */
    /* the emitters' BLAS in LDS (S.sbRecN > 0): after the stack and the tables, 16-B aligned */
    const size_t stgLds = ((((size_t)sw * sizeof(uint16_t) + (size_t)c->nInstances * (sizeof(TraceInst) + sizeof(uint32_t))) + 15) & ~(size_t)15) +
                          (size_t)c->S.sbRecN * 64 + (size_t)c->S.sbTriN * 48;
    /* staged only where the copy still leaves 5 workgroups of 256 per CU
     * (k_connect's residency; 144 B of static LDS each) */
    const bool stg = ldsC && !c->S.laneW && c->S.sbRecN > 0u && (stgLds + 256) * 5 <= 163840;
    c->connectStaged = stg;
    auto connectK = c->S.laneW ? (ldsC ? k_connect<true, true> : k_connect<false, true>)
                               : (ldsC ? (stg ? k_connect<true, false, true> : k_connect<true, false>) : k_connect<false, false>);
    /* staged: 16-bit stack entries (half the stack's LDS) leave room for the
     * copy beside 5 workgroups of 256 per CU, the residency k_connect runs at */
    const size_t connectLds = (!ldsC ? (size_t)sw * sizeof(uint32_t) : stg ? stgLds : traversalLds(c, kBlock)) + c->conLdsPad;
    hipLaunchKernelGGL(connectK, dim3(c->gridConnect), dim3(kBlock), connectLds, s1, c->S, c->Q, c->rad, c->ctr, par, sw);
    if (ovl) (void)hipEventRecord(c->capEv[2 * ph + 1], s1);
    if (ev) (void)hipEventRecord(ev[5], s0);
    if (!c->regenFirst) regen();
}

/* The resume records of the capped lane walk, before the first phase that
 * may write them: one per pool slot (every ray of a phase may stop once) */
int ensureResume(surf_ctx* c) {
    if (!laneCapOn(c) || c->resumeRec) return SURF_OK;
    c->resumeCap = c->capacity;
    return devAlloc(c, c->wfAllocs, &c->resumeRec, (size_t)c->resumeCap * 64u);
}

int buildGraph(surf_ctx* c) {
    if (c->graphExec) return SURF_OK;
    if (int rc = ensureResume(c)) return rc;
    for (int shortG = 0; shortG < 2; ++shortG) {
        SURF_CHECK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        const int nph = shortG ? kPhasesShort : kPhasesPerGraph;
        for (int ph = 0; ph < nph; ++ph) launchPhase(c, ph, nullptr);
        if (c->overlap) (void)hipStreamWaitEvent(c->stream, c->capEv[2 * (nph - 1) + 1], 0);   /* join the last connect */
        hipGraph_t& g = shortG ? c->graphShort : c->graph;
        hipError_t e = hipStreamEndCapture(c->stream, &g);
        if (e != hipSuccess) return fail(c, SURF_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(e));
        SURF_CHECK(c, hipGraphInstantiate(shortG ? &c->graphExecShort : &c->graphExec, g, nullptr, nullptr, 0));
    }
    return SURF_OK;
}

/* Pixel classes of the issue order (cached until the camera, the scene or
 * the instances change): class A = the local pixels whose centre camera ray
 * first hits one of the heavy instances (setKeys).  Long Russian-roulette
 * paths start there (C3 frame 2: 67 % of the paths longer than 100 segments
 * from 4.3 % of the pixels, the two Suzannes); issuing those samples first
 * gives their paths more wavefront phases before the drain takes the
 * survivors.  Only the issue order changes: each sample is the same function
 * of (pixel, frame) and frames are still accumulated in order. */
int classifyPixels(surf_ctx* c) {
    if (c->permValid) return SURF_OK;
    const uint32_t n = c->npx;
    std::vector<float> o(3 * (size_t)n), d(3 * (size_t)n);
    const DevCamera& k = c->cam;
    for (uint32_t lp = 0; lp < n; ++lp) {
        const uint32_t x = lp % c->width, row = c->rows[lp / c->width];
        const float u = (float)x * k.invW, v = (float)row * k.invH;
        float dir[3], len2 = 0.0f;
        for (int a = 0; a < 3; ++a) {
            dir[a] = k.firstPixel[a] + u * k.uVec[a] + v * k.vVec[a] - k.pos[a];
            len2 += dir[a] * dir[a];
        }
        const float inv = 1.0f / std::sqrt(len2);
        for (int a = 0; a < 3; ++a) { o[3 * (size_t)lp + a] = k.pos[a]; d[3 * (size_t)lp + a] = dir[a] * inv; }
    }
    std::vector<void*> tmp;
    float *dO, *dD; float4* dT; uint2* dI;
    int rc;
    if ((rc = devAlloc(c, tmp, &dO, 3 * (size_t)n)) || (rc = devAlloc(c, tmp, &dD, 3 * (size_t)n)) ||
        (rc = devAlloc(c, tmp, &dT, n)) || (rc = devAlloc(c, tmp, &dI, n))) { freeList(tmp); return rc; }
    std::vector<uint2> ip(n);
    (void)hipMemcpyAsync(dO, o.data(), 12 * (size_t)n, hipMemcpyHostToDevice, c->stream);
    (void)hipMemcpyAsync(dD, d.data(), 12 * (size_t)n, hipMemcpyHostToDevice, c->stream);
    hipLaunchKernelGGL(c->S.laneW ? (c->ldsTables ? k_trace_closest<true, true> : k_trace_closest<false, true>)
                                  : (c->ldsTables ? k_trace_closest<true, false> : k_trace_closest<false, false>),
                       dim3((n + kBlock - 1) / kBlock), dim3(kBlock), traversalLds(c, kBlock), c->stream,
                       c->S, (const float*)dO, (const float*)dD, n, dT, dI, stackWords(c, kBlock));
    (void)hipMemcpyAsync(ip.data(), dI, sizeof(uint2) * (size_t)n, hipMemcpyDeviceToHost, c->stream);
    const hipError_t e = hipStreamSynchronize(c->stream);
    freeList(tmp);
    if (e != hipSuccess) return fail(c, SURF_ERR_HIP, std::string("pixel classification: ") + hipGetErrorString(e));
    std::vector<uint32_t> perm;
    perm.reserve(n);
    for (int cls = 0; cls < 2; ++cls)
        for (uint32_t lp = 0; lp < n; ++lp) {
            const bool heavy = std::find(c->heavyInst.begin(), c->heavyInst.end(), ip[lp].x) != c->heavyInst.end();
            if (heavy == (cls == 0)) perm.push_back(lp);
        }
    c->permA = (uint32_t)std::count_if(ip.begin(), ip.end(), [&](const uint2& h) {
        return std::find(c->heavyInst.begin(), c->heavyInst.end(), h.x) != c->heavyInst.end();
    });
    SURF_CHECK(c, hipMemcpy(c->dPerm, perm.data(), sizeof(uint32_t) * (size_t)n, hipMemcpyHostToDevice));
    c->permValid = true;
    return SURF_OK;
}

/* ---- sample stream ------------------------------------------------------ */
int startStream(surf_ctx* c, uint64_t baseFrame, uint32_t maxSeg, uint32_t frames, uint32_t spp) {
    Counters h{};
    for (uint32_t& v : h.capped) v = kUnset;
    /* a multi-frame request that fits the window: its pixels in class order */
    c->permFrames = 0;
    if (c->reorder && frames >= 2 && (uint64_t)frames * spp <= c->window && c->heavyInst.size()) {
        int rc = classifyPixels(c);
        if (rc) return rc;
        if (c->permA > 0 && c->permA < c->npx) c->permFrames = frames;
    }
    h.permFrames = c->permFrames;
    h.permA = c->permFrames ? c->permA : 0u;
    h.maxSeg = maxSeg;
    /* automatic: on for 1-sample frames (radiance-neutral); off for
     * multi-sample frames, whose next sample starts from the RNG state the
     * reference's path ends with -- which an early end would change */
    h.zeroCutoff = (c->zeroCutoff < 0 ? spp == 1 : c->zeroCutoff != 0) ? 1u : 0u;
    h.spp = spp;
    h.baseFrame = baseFrame;
    h.survCap = c->survCap;
    *c->hctr = h;
    SURF_CHECK(c, hipMemcpyAsync(c->ctr, c->hctr, sizeof(Counters), hipMemcpyHostToDevice, c->stream));
    SURF_CHECK(c, hipMemsetAsync(c->frameDone, 0, (size_t)kStripes * c->window * sizeof(uint32_t), c->stream));
    SURF_CHECK(c, hipMemsetAsync(c->Q.cur, 0, (size_t)2 * kShSegs * kShStride * sizeof(uint32_t), c->stream));
    c->streamActive = true;
    c->baseFrame = baseFrame;
    c->targetFrames = 0;
    c->accPasses = 0;
    c->spp = spp;
    c->streamMaxSeg = maxSeg;
    c->pushedLimit = 0;
    c->issuePerPhase = 0;          /* predicted from this stream's own replays only */
    return SURF_OK;
}

/* Chains (first samples of (frame, pixel)) that may be issued: a frame is
 * issued only when all its passes fit the window past the accumulated ones. */
uint64_t issueLimit(const surf_ctx* c) {
    return std::min<uint64_t>(c->targetFrames, (c->accPasses + c->window) / c->spp) * (uint64_t)c->npx;
}
uint64_t targetPasses(const surf_ctx* c) { return c->targetFrames * c->spp; }

int pushLimit(surf_ctx* c) {
    const uint64_t lim = issueLimit(c);
    if (lim == c->pushedLimit) return SURF_OK;
    uint64_t* src = &c->hLimit[c->hLimitNext++ % surf_ctx::kLimitRing];
    *src = lim;
    SURF_CHECK(c, hipMemcpyAsync(&c->ctr->limit, src, sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
    c->pushedLimit = lim;
    return SURF_OK;
}

/* Frames whose every chain is issued after `iss` chains (k_regen's order:
 * the permuted head of permFrames frames, then frame-major). */
uint64_t fullyIssuedFrames(const surf_ctx* c, uint64_t iss) {
    const uint64_t P = c->permFrames;
    if (!P || iss >= (uint64_t)c->npx * P) return iss / c->npx;
    const uint64_t endA = (uint64_t)c->permA * P;
    return iss <= endA ? 0 : (iss - endA) / (c->npx - c->permA);
}

/* Finished paths of a frame slot in a snapshot: sum over the completion stripes. */
uint64_t framePaths(const surf_ctx* c, const uint32_t* fd, uint32_t slot) {
    uint64_t n = 0;
    for (uint32_t k = 0; k < kStripes; ++k) n += fd[(size_t)k * c->window + slot];
    return n;
}

/* Event totals of the current stream: plain counters + the block stripes. */
void streamEvents(const Counters& h, unsigned long long out[kEvents]) {
    for (int k = 0; k < kEvents; ++k) {
        out[k] = h.ev[k];
        for (uint32_t s = 0; s < kStripes; ++s) out[k] += h.evS[s][k];
    }
}

/* Queues a snapshot of the counters and of the open passes' completion
 * stripes ([accPasses, targetPasses), at most a window: a strided copy of
 * their slots in each stripe row), taken after `replays` graph replays. */
int enqueueSnap(surf_ctx* c, int phases) {
    surf_ctx::Snap& sn = c->snap[(c->snapHead + c->snapCount) % surf_ctx::kSnaps];
    SURF_CHECK(c, hipMemcpyAsync(sn.h, c->ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    const uint64_t tp = targetPasses(c);
    const uint64_t open = std::min<uint64_t>(tp - std::min(c->accPasses, tp), c->window);
    const uint32_t s0 = (uint32_t)(c->accPasses % c->window);
    const uint32_t n0 = (uint32_t)std::min<uint64_t>(open, c->window - s0);
    const size_t pitch = (size_t)c->window * sizeof(uint32_t);
    if (n0)
        SURF_CHECK(c, hipMemcpy2DAsync(sn.fd + s0, pitch, c->frameDone + s0, pitch, n0 * sizeof(uint32_t), kStripes,
                                       hipMemcpyDeviceToHost, c->stream));
    if (open > n0)
        SURF_CHECK(c, hipMemcpy2DAsync(sn.fd, pitch, c->frameDone, pitch, (open - n0) * sizeof(uint32_t), kStripes,
                                       hipMemcpyDeviceToHost, c->stream));
    SURF_CHECK(c, hipEventRecord(sn.ev, c->stream));
    sn.acc = c->accPasses;
    sn.open = open;
    sn.phases = phases;
    ++c->snapCount;
    return SURF_OK;
}

/* Waits for the oldest snapshot, makes it the host's view of the counters and
 * accumulates, in pass order, every leading pass whose samples have all
 * finished in it.  A pass is complete when all its samples were issued and
 * all finished; a slot is reused only after its pass is accumulated, so passes
 * of frames not yet fully issued must not be tested (their slot may still
 * count an older pass), nor passes past the snapshot's copied range.  Later
 * replays already queued cannot touch the slots accumulated here: the issue
 * limit they run under was pushed before this accumulation. */
int consumeSnap(surf_ctx* c) {
    surf_ctx::Snap& sn = c->snap[c->snapHead];
    SURF_CHECK(c, hipEventSynchronize(sn.ev));
    const uint64_t before = c->hctr->issued[0];
    std::memcpy(c->hctr, sn.h, sizeof(Counters));
    /* per phase (a replay is kPhasesPerGraph or kPhasesShort phases), and only from a replay
     * that issued under its limit the whole time: a starved one undercounts */
    if (sn.phases > 0 && c->hctr->issued[0] > before && c->hctr->issued[0] < c->hctr->limit)
        c->issuePerPhase = (c->hctr->issued[0] - before) / (uint64_t)sn.phases;
    c->snapHead = (c->snapHead + 1) % surf_ctx::kSnaps;
    --c->snapCount;
    for (int k = 0; k < 2; ++k)                       /* calls whose end this snapshot has passed */
        if (c->tevPending[k] && hipEventQuery(c->tev[k][1]) == hipSuccess) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, c->tev[k][0], c->tev[k][1]);
            c->stats.ms_total += ms;
            c->tevPending[k] = false;
        }
    const uint64_t tp = targetPasses(c);
    const uint64_t issuedPasses = fullyIssuedFrames(c, c->hctr->issued[0]) * c->spp;
    const uint64_t hi = sn.acc + sn.open;
    uint64_t f = c->accPasses;
    while (f < tp && f < issuedPasses && f < hi && framePaths(c, sn.fd, (uint32_t)(f % c->window)) == c->npx) ++f;
    if (f == c->accPasses) return SURF_OK;
    const uint32_t count = (uint32_t)(f - c->accPasses);
    const uint32_t threads = std::max<uint32_t>(c->npx, count * kStripes);
    hipLaunchKernelGGL(k_accumulate, dim3((threads + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream, (const float4*)c->rad,
                       c->acc, c->npx, (unsigned long long)c->accPasses, count, c->window, c->frameDone);
    SURF_CHECK(c, hipGetLastError());
    c->accPasses = f;
    return pushLimit(c);
}

int consumeAll(surf_ctx* c) {
    int rc;
    while (c->snapCount)
        if ((rc = consumeSnap(c))) return rc;
    return SURF_OK;
}

/* Reads counters + per-pass completion (one sync) and accumulates. */
int syncAndAccumulate(surf_ctx* c, int phases = 0) {
    int rc;
    if ((rc = consumeAll(c)) || (rc = enqueueSnap(c, phases))) return rc;
    return consumeSnap(c);
}

/* One unit of forward progress: kPhasesPerGraph phases (graph replay, or
 * direct launches with per-kernel events when profiling). */
int advance(surf_ctx* c, bool shortRun = false) {
    const int phases = shortRun ? kPhasesShort : kPhasesPerGraph;
    if (c->profiling) {
        if (int rc = ensureResume(c)) return rc;
        for (int ph = 0; ph < phases; ++ph) launchPhase(c, ph, &c->pev[kPhaseEvents * ph]);
        SURF_CHECK(c, hipEventRecord(c->pev[kPhaseEvents * phases], c->stream));
        SURF_CHECK(c, hipGetLastError());
        SURF_CHECK(c, hipEventSynchronize(c->pev[kPhaseEvents * phases]));
        for (int ph = 0; ph < phases; ++ph) {
            float t[kPhaseEvents];
            for (int k = 0; k < kPhaseEvents; ++k)
                (void)hipEventElapsedTime(&t[k], c->pev[kPhaseEvents * ph + k], c->pev[kPhaseEvents * ph + k + 1]);
            /* (t[3]: k_regen when it runs before the fork, else nothing) */
            c->stats.ms_sort += t[0];
            c->stats.ms_extend += t[1]; c->stats.ms_shade += t[2]; c->stats.ms_connect += t[4]; c->stats.ms_regen += t[3] + t[5];
            c->stats.launches_extend++;
            if (c->phaseLog)
                std::fprintf(c->phaseLog, "phase %u sort %.4f extend %.4f shade %.4f regen %.4f connect %.4f\n", c->hPhaseN[ph], t[0], t[1],
                             t[2], t[3] + t[5], t[4]);
        }
        if (c->phaseLog) std::fflush(c->phaseLog);
    } else {
        SURF_CHECK(c, hipGraphLaunch(shortRun ? c->graphExecShort : c->graphExec, c->stream));
    }
    c->stats.iterations += phases;
    if (c->stats.iterations > kMaxIterations)
        return fail(c, SURF_ERR_LIMIT, "wavefront did not drain after " + std::to_string(c->stats.iterations) + " iterations");
    return SURF_OK;
}

/* Finishes every path of pool 0 in one k_tail launch (counters at an even
 * phase boundary: pool 0 is the next to be extended, nothing else pending). */
void launchTail(surf_ctx* c, Pool in, uint32_t n, uint32_t lpw, uint32_t firstCounted, uint32_t budget, Pool out) {
    const uint32_t blocks = (n + lpw - 1) / lpw;
    const size_t lds = traversalLds(c, 64);
    if (c->ldsTables)
        hipLaunchKernelGGL(k_tail<true>, dim3(blocks), dim3(64), lds, c->stream, c->S, in, n, lpw, c->rad, c->frameDone,
                           c->npx, c->window, c->ctr, stackWords(c, 64), firstCounted, budget, out, c->cam, geom(c));
    else
        hipLaunchKernelGGL(k_tail<false>, dim3(blocks), dim3(64), lds, c->stream, c->S, in, n, lpw, c->rad, c->frameDone,
                           c->npx, c->window, c->ctr, stackWords(c, 64), firstCounted, budget, out, c->cam, geom(c));
}

/* Finishes every path of pool 0 (counters at an even phase boundary: pool 0 is
 * the next to be extended, nothing else pending).  Lane-parallel stages (many
 * paths per wave) run each path for up to tailBudget segments and hand the
 * paths still alive to the next stage; once few enough remain (they are the
 * reference's Russian-roulette survivors that run for thousands of segments),
 * the cooperative tail runs each on a whole wave, which cuts the latency of a
 * segment -- the quantity the last paths of a drain are bound by. */
/* The cooperative drain uses the lanes-as-planes wave traversal (traceWave):
 * single-leaf TLAS of <= 64 instances, stack of node records in 64 lanes. */
/* Any TLAS (traceWaveTlas walks one whose root splits or that holds > 64
 * instances); the TLAS stack is one VGPR (<= 64 entries). */
bool waveEligible(const surf_ctx* c) { return c->hasScene && c->stackDepth <= 64 && coopLdsOk(c); }

/* Regen counted each pool-0 path's next extension ray (firstCounted). */
int runTail(surf_ctx* c) {
    const uint32_t n = c->hctr->nIn[0];
    if (n == 0) return SURF_OK;
    if (c->profiling) SURF_CHECK(c, hipEventRecord(c->pev[0], c->stream));
    Pool in = c->pool[0];
    uint32_t cnt = n, firstCounted = 1u;
    c->tailFirstRays += n;
    int buf = 0;
    static const bool dbg = std::getenv("SURF_DEBUG_TAIL") != nullptr;   /* diagnostics: per-stage log on stderr */
    auto t0 = std::chrono::steady_clock::now();
    for (int stage = 0; cnt; ++stage) {
        if (dbg) {
            SURF_CHECK(c, hipStreamSynchronize(c->stream));
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            std::fprintf(stderr, "[surf tail] stage %d: %u paths at %.2f ms\n", stage, cnt, ms);
        }
        if (c->tailPair && waveEligible(c) && cnt <= c->coopAll) {
            /* as many two-wave workgroups as are resident at once, each wave
             * taking paths from the queue; idle waves trace their sibling's
             * shadow rays once the queue is empty */
            int per = 0;
            const bool w2 = c->S.wnodes != nullptr;
            auto kern = c->ldsTables ? (w2 ? k_tail_pair<true, true> : k_tail_pair<true, false>)
                                     : (w2 ? k_tail_pair<false, true> : k_tail_pair<false, false>);
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, 128, pairTailLds(c)) != hipSuccess || per < 1)
                per = 2 * SURF_COOP_WAVES;
            const uint32_t blocks = std::max<uint32_t>(1u, std::min<uint32_t>((cnt + 1u) / 2u, c->cus * (uint32_t)per));
            SURF_CHECK(c, hipMemsetAsync(&c->ctr->rowNext, 0, sizeof(uint32_t), c->stream));
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(128), pairTailLds(c), c->stream, c->S, in, cnt, c->rad, c->frameDone,
                               c->npx, c->window, c->ctr, recStackWords(c), firstCounted, c->cam, geom(c));
            SURF_CHECK(c, hipGetLastError());
            c->stats.tail_survivors += cnt;
            break;
        }
        if (waveEligible(c) && cnt <= c->coopAll) {
            const bool w2 = c->S.wnodes != nullptr;
            hipLaunchKernelGGL(c->ldsTables ? (w2 ? k_tail_coop<true, true> : k_tail_coop<true, false>)
                                            : (w2 ? k_tail_coop<false, true> : k_tail_coop<false, false>),
                               dim3(cnt), dim3(64), coopTailLds(c), c->stream,
                               c->S, in, cnt, c->rad, c->frameDone,
                               c->npx, c->window, c->ctr, recStackWords(c), firstCounted, c->cam, geom(c));
            SURF_CHECK(c, hipGetLastError());
            c->stats.tail_survivors += cnt;
            break;
        }
        /* no more waves than fit at once (2 per SIMD at the tail's register
         * count): a second round would wait for the first round's longest path */
        const uint32_t lpw = c->tailLanes ? std::min<uint32_t>(64u, c->tailLanes)
                                          : std::min<uint32_t>(64u, std::max<uint32_t>(1u, (cnt + c->coopMax - 1) / c->coopMax));
        c->hctr->survN = 0;
        SURF_CHECK(c, hipMemcpyAsync(&c->ctr->survN, &c->hctr->survN, sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
        launchTail(c, in, cnt, lpw, firstCounted, c->tailBudget, c->surv[buf]);
        SURF_CHECK(c, hipGetLastError());
        if (!c->tailBudget) break;
        SURF_CHECK(c, hipMemcpyAsync(&c->hctr->survN, &c->ctr->survN, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
        SURF_CHECK(c, hipStreamSynchronize(c->stream));
        in = c->surv[buf];
        cnt = std::min(c->hctr->survN, c->survCap);
        firstCounted = 0u;
        buf ^= 1;
    }
    if (c->profiling) {
        SURF_CHECK(c, hipEventRecord(c->pev[1], c->stream));
        SURF_CHECK(c, hipEventSynchronize(c->pev[1]));
        float t; (void)hipEventElapsedTime(&t, c->pev[0], c->pev[1]);
        c->stats.ms_tail += t;
    }
#if SURF_DRAIN_TRACE
    if (const char* path = std::getenv("SURF_DRAIN_TRACE_FILE")) {
        /* diagnostics: one line per path the cooperative drain finished */
        SURF_CHECK(c, hipStreamSynchronize(c->stream));
        uint32_t nrec = 0;
        SURF_CHECK(c, hipMemcpyFromSymbol(&nrec, HIP_SYMBOL(g_drainEndN), sizeof nrec));
        nrec = std::min(nrec, kDrainTraceCap);
        std::vector<uint4> rec(nrec);
        if (nrec) SURF_CHECK(c, hipMemcpyFromSymbol(rec.data(), HIP_SYMBOL(g_drainEnd), nrec * sizeof(uint4)));
        int khz = 0;
        (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device);
        if (FILE* f = std::fopen(path, "a")) {
            std::fprintf(f, "# drain %u paths, clock %d kHz: end_lo state segments start_lo\n", n, khz);
            for (const uint4& r : rec) std::fprintf(f, "%u %u %u %u\n", r.x, r.y, r.z, r.w);
            std::fclose(f);
        }
        const uint32_t zero = 0;
        SURF_CHECK(c, hipMemcpyToSymbol(HIP_SYMBOL(g_drainEndN), &zero, sizeof zero));
    }
#endif
#if SURF_SEG_TIMING
    if (dbg) {
        SURF_CHECK(c, hipMemcpyAsync(c->hctr, c->ctr, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
        SURF_CHECK(c, hipStreamSynchronize(c->stream));
        const unsigned long long* g = c->hctr->dbg;
        const double ns = (double)std::max(1ull, g[3]);
        std::fprintf(stderr, "[surf tail] coop cycles per segment: extend %.0f shade %.0f connect %.0f (%llu segments, %llu shadow)\n",
                     g[0] / ns, g[1] / ns, g[2] / ns, g[3], g[4]);
        unsigned long long h[8];
        SURF_CHECK(c, hipMemcpyFromSymbol(h, HIP_SYMBOL(g_segStats), sizeof(h)));
        std::fprintf(stderr, "[surf tail] extend per segment: instance prologues %.0f cycles, BLAS loops %.0f cycles, %.1f interior visits, "
                     "%.1f leaves, %.1f triangles, %.2f instances entered; %.0f cycles waiting for prefetched records, %.0f in leaves\n",
                     h[0] / ns, h[1] / ns, h[2] / ns, h[3] / ns, h[4] / ns, h[5] / ns, h[6] / ns, h[7] / ns);
        const unsigned long long zero[8] = {};
        SURF_CHECK(c, hipMemcpyToSymbol(HIP_SYMBOL(g_segStats), zero, sizeof(zero)));   /* per drain, like the counters */
    }
#endif
    /* pool 0 is now empty: the next phase starts from regen's refill */
    c->hctr->nIn[0] = 0;
    SURF_CHECK(c, hipMemcpyAsync(&c->ctr->nIn[0], &c->hctr->nIn[0], sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    return SURF_OK;
}

/* Drain hand-over (automatic): a quarter frame of paths (W * H / 4, what
 * capacity / 16 was at the round-2 pool of 4 frames), at most capacity / 16:
 * tied to the pool, a larger pool handed C5's deep-BVH drain 280 k paths
 * (drain 2.2 -> 5.8 s per render). */
uint32_t tailThreshold(const surf_ctx* c) {
    if (c->tailPaths) return c->tailPaths;
    const uint64_t quarter = (uint64_t)c->width * c->height / 4;
    return (uint32_t)std::max<uint64_t>(std::min<uint64_t>(quarter, c->capacity / 16), 4096u);
}

/* Runs until every requested sample is issued (drain = false) or until every
 * requested frame is accumulated (drain = true).  While issuing, a call runs
 * pipelined: it queues the next replay before it has read the previous one's
 * counters -- predicting what the replays in flight issue -- and may return
 * with up to kSnaps replays in flight, so the GPU does not wait for the host
 * between polls or calls (the drop-in loop's one-frame calls).  Drains, the
 * tail and a starved stream decide from fresh counters. */
int pump(surf_ctx* c, bool drain, uint64_t lag) {
    int rc;
    const bool pipe = c->pipeline && !drain;
    if (!pipe && (rc = consumeAll(c))) return rc;
    if ((rc = pushLimit(c))) return rc;
    const uint64_t target = c->targetFrames * (uint64_t)c->npx;
    for (;;) {
        if (pipe)       /* the snapshots that have landed, and the oldest when both are in flight */
            while (c->snapCount && (c->snapCount == surf_ctx::kSnaps || hipEventQuery(c->snap[c->snapHead].ev) == hipSuccess))
                if ((rc = consumeSnap(c))) return rc;
        const uint64_t issued = c->hctr->issued[0];
        /* what the replays in flight issue: predicted per phase, never past the pushed limit */
        uint64_t inflightPhases = 0;
        for (int k = 0; k < c->snapCount; ++k) inflightPhases += (uint64_t)c->snap[(c->snapHead + k) % surf_ctx::kSnaps].phases;
        const uint64_t ahead = std::min<uint64_t>(inflightPhases * c->issuePerPhase, c->pushedLimit - std::min(issued, c->pushedLimit));
        /* in flight at a replay boundary: the pool the next phase extends */
        const uint32_t inflight = c->hctr->nIn[0];
        if (!drain && issued + ahead + lag >= target) return SURF_OK;
        if (drain && c->accPasses >= targetPasses(c)) return SURF_OK;
        const bool starved = issued >= c->pushedLimit;     /* nothing more may be issued right now */
        if (c->snapCount && starved) {                     /* decided from fresh counters */
            if ((rc = consumeAll(c))) return rc;
            continue;
        }
        const uint64_t accBefore = c->accPasses;
        static const bool dbgDrain = std::getenv("SURF_DEBUG_DRAIN") != nullptr;   /* diagnostics: drain timeline */
        if (dbgDrain && starved) {
            static auto tS = std::chrono::steady_clock::now();
            std::fprintf(stderr, "[surf drain] iteration %llu: %u paths in flight, %llu/%llu passes at %.3f ms\n",
                         (unsigned long long)c->stats.iterations, inflight, (unsigned long long)c->accPasses,
                         (unsigned long long)targetPasses(c),
                         std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tS).count());
        }
        int phases = 0;
        if (starved && inflight > 0 && inflight <= tailThreshold(c)) {
            if ((rc = runTail(c))) return rc;
        } else if (starved && inflight == 0) {
            /* every issued sample finished: accumulating re-opens the window */
        } else {
            /* draining (nothing left to issue): several replays per host poll --
             * the per-replay poll, not the kernels, is what a small pool pays */
            const int reps = starved ? c->drainReplays : 1;
            /* a per-frame render call (lagged, or at most one frame left to
             * issue): short replays (SURF_DRAIN_SHORT=1: also once nothing is
             * left to issue, so the drain takes over within kPhasesShort phases instead
             * of up to 8 -- measured slower) */
            const bool shortRun = (!drain && (lag > 0 || target - issued <= c->npx)) || (starved && c->drainShort);
            for (int k = 0; k < reps; ++k)
                if ((rc = advance(c, shortRun))) return rc;
            phases = reps * (shortRun ? kPhasesShort : kPhasesPerGraph);
            if (pipe) {                                    /* read later: queue the next replay first */
                if ((rc = enqueueSnap(c, phases))) return rc;
                continue;
            }
        }
        if ((rc = syncAndAccumulate(c, phases))) return rc;
        if (starved && inflight == 0 && c->accPasses == accBefore)
            return fail(c, SURF_ERR_HIP, "sample stream stalled: pool empty but frames incomplete");
    }
}

/* Adds the device time of calls that returned with replays in flight (their
 * ends have passed once the stream is idle). */
void collectCallTimes(surf_ctx* c) {
    for (int k = 0; k < 2; ++k)
        if (c->tevPending[k]) {
            (void)hipEventSynchronize(c->tev[k][1]);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, c->tev[k][0], c->tev[k][1]);
            c->stats.ms_total += ms;
            c->tevPending[k] = false;
        }
}

int ensureDrained(surf_ctx* c) {
    if (!c->streamActive) return SURF_OK;
    SURF_CHECK(c, hipSetDevice(c->device));
    {
        const int rc = consumeAll(c);                 /* the host's counters as of the last replay */
        if (rc) return rc;
        collectCallTimes(c);
    }
    if (c->accPasses >= targetPasses(c)) return SURF_OK;
    if (!c->profiling) {
        int rc = buildGraph(c);
        if (rc) return rc;
    }
    SURF_CHECK(c, hipEventRecord(c->ev0, c->stream));
    int rc = pump(c, true, 0);
    if (rc) return rc;
    SURF_CHECK(c, hipEventRecord(c->ev1, c->stream));
    SURF_CHECK(c, hipEventSynchronize(c->ev1));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev0, c->ev1);
    c->stats.ms_total += ms;
    return SURF_OK;
}

/* A stream ends when its pool is empty and all its frames are accumulated. */
int endStream(surf_ctx* c) {
    int rc = ensureDrained(c);
    if (rc) return rc;
    if (c->streamActive) {
        unsigned long long e[kEvents];
        streamEvents(*c->hctr, e);
        for (int k = 0; k < kEvents; ++k) c->evBase[k] += e[k];
        c->segMaxBase = std::max(c->segMaxBase, c->hctr->segMax);
    }
    c->streamActive = false;
    return SURF_OK;
}

/* Which rows a shard owns. */
std::vector<uint32_t> shardRows(uint32_t height, uint32_t shard, uint32_t shards, uint32_t block) {
    std::vector<uint32_t> rows;
    if (block == 0) {
        const uint32_t r0 = (uint32_t)((uint64_t)height * shard / shards), r1 = (uint32_t)((uint64_t)height * (shard + 1) / shards);
        for (uint32_t r = r0; r < r1; ++r) rows.push_back(r);
    } else {
        for (uint32_t r = 0; r < height; ++r)
            if ((r / block) % shards == shard) rows.push_back(r);
    }
    return rows;
}

int createCtx(int dev, uint32_t w, uint32_t h, std::vector<uint32_t> rows, surf_ctx** out) {
    if (!out) return fail(nullptr, SURF_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (w == 0 || h == 0 || rows.empty()) return fail(nullptr, SURF_ERR_INVALID, "empty frame or shard");
    if ((uint64_t)w * rows.size() > (1ull << 31)) return fail(nullptr, SURF_ERR_INVALID, "shard too large");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || dev < 0 || dev >= count) return fail(nullptr, SURF_ERR_NO_DEVICE, "no HIP device " + std::to_string(dev));
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(nullptr, SURF_ERR_NO_DEVICE, "hipGetDeviceProperties failed");
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return fail(nullptr, SURF_ERR_NO_DEVICE, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950");
    /* tuning knobs (A/B runs): read once per context, invalid values refused */
    uint32_t extBlock = 128;
    if (const char* e = std::getenv("SURF_EXTEND_BLOCK")) {
        const int b = std::atoi(e);
        if (b != 128 && b != 256) return fail(nullptr, SURF_ERR_INVALID, std::string("SURF_EXTEND_BLOCK must be 128 or 256, not ") + e);
        extBlock = (uint32_t)b;
    }
    auto* c = new surf_ctx();
    c->device = dev;
    c->extBlock = extBlock;
    if (const char* e = std::getenv("SURF_SORT")) {
        c->sortRays = e[0] != '0';
        c->sortPool = e[0] != '3';
        c->sortShadow = e[0] != '2';
    }
    if (const char* e = std::getenv("SURF_CONNECT_GLOBAL")) c->connectGlobal = e[0] != '0';
    if (const char* e = std::getenv("SURF_EXT_STACK16")) c->extStack16 = e[0] != '0';
    if (const char* e = std::getenv("SURF_REGEN_COUNT")) c->regenCount = e[0] != '0';
    if (const char* e = std::getenv("SURF_LANE_CAP")) c->laneCap = (uint32_t)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("SURF_KEY")) c->keyMode = e[0] == '0' ? 0u : (e[0] == '1' ? 1u : 2u);
    if (const char* e = std::getenv("SURF_OVERLAP")) c->overlap = e[0] != '0';
    if (const char* e = std::getenv("SURF_LOOP_LAG")) c->loopLag = e[0] != '0';
    if (const char* e = std::getenv("SURF_EXT_LDS_PAD")) c->extLdsPad = (size_t)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("SURF_CON_LDS_PAD")) c->conLdsPad = (size_t)std::max(0, std::atoi(e));
    if (const char* e = std::getenv("SURF_LDS_LIGHTBLAS")) c->ldsLightBlas = e[0] != '0';
    if (const char* e = std::getenv("SURF_REORDER")) c->reorder = e[0] != '0';
    if (const char* e = std::getenv("SURF_TAIL_PAIR")) c->tailPair = e[0] != '0';
    if (const char* e = std::getenv("SURF_DRAIN_SHORT")) c->drainShort = e[0] == '1';
    if (const char* e = std::getenv("SURF_REGEN_FIRST")) c->regenFirst = e[0] == '1';
    if (const char* e = std::getenv("SURF_PIPELINE")) c->pipeline = e[0] != '0';
    c->width = w;
    c->height = h;
    c->rows = std::move(rows);
    c->npx = (uint32_t)(w * c->rows.size());
    if (hipSetDevice(dev) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail(nullptr, SURF_ERR_HIP, "stream/event creation failed");
    }
    for (auto& e : c->capEv)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
            delete c;
            return fail(nullptr, SURF_ERR_HIP, "event creation failed");
        }
    if (hipMalloc(&c->acc, (size_t)c->npx * sizeof(float4)) != hipSuccess ||
        hipMalloc(&c->dRows, c->rows.size() * sizeof(uint32_t)) != hipSuccess) {
        surf_destroy(c);
        return fail(nullptr, SURF_ERR_OOM, "accumulator allocation failed");
    }
    (void)hipMemset(c->acc, 0, (size_t)c->npx * sizeof(float4));
    (void)hipMemcpy(c->dRows, c->rows.data(), c->rows.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    *out = c;
    return SURF_OK;
}

}  // namespace

extern "C" {

int surf_abi_version(void) { return SURF_ABI_VERSION; }

int surf_device_count(int* count) {
    if (!count) return SURF_ERR_INVALID;
    *count = 0;
    if (hipGetDeviceCount(count) != hipSuccess) { *count = 0; return fail(nullptr, SURF_ERR_NO_DEVICE, "hipGetDeviceCount failed"); }
    return SURF_OK;
}

int surf_create(int dev, uint32_t w, uint32_t h, uint32_t r0, uint32_t r1, surf_ctx** out) {
    if (r0 >= r1 || r1 > h) return fail(nullptr, SURF_ERR_INVALID, "row range out of frame");
    std::vector<uint32_t> rows;
    for (uint32_t r = r0; r < r1; ++r) rows.push_back(r);
    return createCtx(dev, w, h, std::move(rows), out);
}

int surf_create_sharded(int dev, uint32_t w, uint32_t h, uint32_t shard, uint32_t shards, uint32_t block, surf_ctx** out) {
    if (shards == 0 || shard >= shards) return fail(nullptr, SURF_ERR_INVALID, "bad shard index");
    return createCtx(dev, w, h, shardRows(h, shard, shards, block), out);
}

void surf_destroy(surf_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    destroyGraph(c);
    freeList(c->sceneAllocs);
    freeList(c->wfAllocs);
    if (c->hctr) (void)hipHostFree(c->hctr);
    if (c->hLimit) (void)hipHostFree(c->hLimit);
    for (auto& sn : c->snap) {
        if (sn.h) (void)hipHostFree(sn.h);
        if (sn.fd) (void)hipHostFree(sn.fd);
        if (sn.ev) (void)hipEventDestroy(sn.ev);
    }
    for (auto& pr : c->tev)
        for (auto& e : pr) if (e) (void)hipEventDestroy(e);
    if (c->rad) (void)hipFree(c->rad);
    if (c->frameDone) (void)hipFree(c->frameDone);
    for (auto& e : c->pev) if (e) (void)hipEventDestroy(e);
    if (c->hPhaseN) (void)hipHostFree(c->hPhaseN);
    if (c->phaseLog) std::fclose(c->phaseLog);
    if (c->acc) (void)hipFree(c->acc);
    if (c->dRows) (void)hipFree(c->dRows);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (auto& e : c->capEv)
        if (e) (void)hipEventDestroy(e);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* surf_last_error(const surf_ctx* c) {
    if (c) return c->err.c_str();
    std::lock_guard<std::mutex> l(gErrMutex);
    static thread_local std::string copy;
    copy = gLastError;
    return copy.c_str();
}

int surf_shard_rows(const surf_ctx* c, uint32_t* rows, uint32_t* count) {
    if (!c || !count) return SURF_ERR_INVALID;
    if (rows) std::memcpy(rows, c->rows.data(), c->rows.size() * sizeof(uint32_t));
    *count = (uint32_t)c->rows.size();
    return SURF_OK;
}

int surf_get_device(const surf_ctx* c, int* dev) {
    if (!c || !dev) return SURF_ERR_INVALID;
    *dev = c->device;
    return SURF_OK;
}

int surf_shard_row_list(uint32_t height, uint32_t shard, uint32_t shards, uint32_t block, uint32_t* rows, uint32_t* count) {
    if (!count || shards == 0 || shard >= shards) return fail(nullptr, SURF_ERR_INVALID, "bad shard index");
    const std::vector<uint32_t> r = shardRows(height, shard, shards, block);
    if (rows && !r.empty()) std::memcpy(rows, r.data(), r.size() * sizeof(uint32_t));
    *count = (uint32_t)r.size();
    return SURF_OK;
}

int surf_set_pool_capacity(surf_ctx* c, uint32_t paths) {
    if (!c || paths < 64) return SURF_ERR_INVALID;
    if (c->allocated) return fail(c, SURF_ERR_INVALID, "pool capacity is fixed after the first render");
    c->capacity = paths;
    return SURF_OK;
}

int surf_set_frame_batch(surf_ctx* c, uint32_t frames) {
    if (!c || frames == 0 || (uint64_t)frames * c->npx >= (1ull << 32)) return SURF_ERR_INVALID;
    if (c->allocated) return fail(c, SURF_ERR_INVALID, "frame window is fixed after the first render");
    c->window = frames;
    c->windowFixed = true;
    return SURF_OK;
}

/* Diagnostics: how many paths the segment cap ended in the current stream, and
 * sample ids (slot * npx + shard pixel) of up to 64 of them (unused entries ~0). */
int surf_debug_capped(surf_ctx* c, uint32_t* sids, uint32_t max, uint64_t* count) {
    if (!c || !count) return SURF_ERR_INVALID;
    int rc = ensureDrained(c);
    if (rc) return rc;
    *count = 0;
    if (c->hctr) {
        unsigned long long e[kEvents];
        streamEvents(*c->hctr, e);
        *count = e[7];
    }
    /* the recorded ids: slot blockIdx % 64 of each workgroup that capped a path (racy, any one per slot) */
    uint32_t n = 0;
    if (c->hctr)
        for (uint32_t k = 0; k < 64 && n < max && n < *count; ++k)
            if (c->hctr->capped[k] != kUnset) { if (sids) sids[n] = c->hctr->capped[k]; ++n; }
    if (sids)
        for (uint32_t k = n; k < std::min<uint32_t>(max, 64u); ++k) sids[k] = kUnset;
    return SURF_OK;
}

int surf_debug_issue_order(surf_ctx* c, uint32_t* heavy_pixels, uint32_t* permuted_frames) {
    if (!c || !heavy_pixels || !permuted_frames) return SURF_ERR_INVALID;
    *heavy_pixels = c->permFrames ? c->permA : 0u;
    *permuted_frames = c->permFrames;
    return SURF_OK;
}

int surf_set_tail_policy(surf_ctx* c, uint32_t threshold_paths, uint32_t lanes_per_wave, uint32_t stage_segments) {
    if (!c) return fail(nullptr, SURF_ERR_INVALID, "ctx is NULL");
    if (lanes_per_wave > 64) return fail(c, SURF_ERR_INVALID, "lanes_per_wave must be <= 64");
    SURF_CHECK(c, hipSetDevice(c->device));
    const int rc = endStream(c);
    if (rc) return rc;
    c->tailPaths = threshold_paths;
    c->tailLanes = lanes_per_wave;
    c->tailBudget = stage_segments;
    return SURF_OK;
}

int surf_set_tail_coop(surf_ctx* c, uint32_t max_paths) {
    if (!c) return fail(nullptr, SURF_ERR_INVALID, "ctx is NULL");
    SURF_CHECK(c, hipSetDevice(c->device));
    const int rc = endStream(c);
    if (rc) return rc;
    c->coopAll = max_paths;
    return SURF_OK;
}

int surf_set_trace_mode(surf_ctx* c, int mode) {
    if (!c) return fail(nullptr, SURF_ERR_INVALID, "ctx is NULL");
    if (mode < 0 || mode > 1) return fail(c, SURF_ERR_INVALID, "trace mode must be 0 or 1");
    if (mode == 1 && !waveEligible(c))
        return fail(c, SURF_ERR_INVALID, "one-ray-per-wave traversal needs a BVH stack <= 64 entries");
    c->traceMode = mode;
    return SURF_OK;
}

int surf_set_zero_cutoff(surf_ctx* c, int enabled) {
    if (!c) return SURF_ERR_INVALID;
    int rc = endStream(c);
    if (rc) return rc;
    c->zeroCutoff = enabled < 0 ? -1 : (enabled != 0 ? 1 : 0);
    return SURF_OK;
}

int surf_set_profiling(surf_ctx* c, int enabled) {
    if (!c) return SURF_ERR_INVALID;
    int rc = endStream(c);
    if (rc) return rc;
    c->profiling = enabled != 0;
    return SURF_OK;
}

/* Instance-dependent tables (GPUScene::update re-uploads exactly these,
 * scene.cpp:267-282): DevInstance + TraceInst per instance, the TLAS node
 * records and index array, the light list.  BLAS roots come from the upload. */
struct InstanceTables {
    std::vector<DevInstance> inst;
    std::vector<TraceInst> tinst;
    std::vector<float4> tnodes;
    std::vector<uint32_t> tidx;
    std::vector<uint2> lights;
    uint32_t tlasDepth = 0, tlasLeafCount = 0;
    uint32_t nHeavy = 0;
    float4 hvLo[3], hvHi[3];
    uint32_t hvInst[3] = {0, 0, 0};
};

/* The heavy-instance boxes of the ray-order keys (kernel arguments). */
void setKeys(surf_ctx* c, DevScene& S, const InstanceTables& T) {
    c->heavyInst.assign(T.hvInst, T.hvInst + T.nHeavy);
    c->permValid = false;                 /* the pixel classes follow the instances */
    S.nHeavy = T.nHeavy;
    for (uint32_t h = 0; h < 3; ++h) {
        S.hvLo[h] = h < T.nHeavy ? T.hvLo[h] : make_float4(0, 0, 0, 0);
        S.hvHi[h] = h < T.nHeavy ? T.hvHi[h] : make_float4(0, 0, 0, 0);
    }
    S.keyMode = T.nHeavy ? c->keyMode : 0u;
    /* the emitters' BLAS, when every light instance uses one BLAS and its
     * node records fit kLdsLightBlas bytes: k_connect stages them */
    S.sbNode0 = S.sbRecN = S.sbTri0 = S.sbTriN = 0u;
    S.sbRec = nullptr;
    if (c->ldsLightBlas && !T.lights.empty()) {
        bool one = true;
        const DevInstance* L0 = T.lights[0].x < T.inst.size() ? &T.inst[T.lights[0].x] : nullptr;
        for (const uint2& L : T.lights)
            one = one && L0 && L.x < T.inst.size() && T.inst[L.x].nodeOffset == L0->nodeOffset &&
                  T.inst[L.x].idxOffset == L0->idxOffset && T.inst[L.x].triOffset == L0->triOffset;
        const auto sb = one ? c->stagedBlas.find(L0->nodeOffset) : c->stagedBlas.end();
        /* 16-bit stack entries: every BLAS and TLAS node index below 65536 */
        const bool small = c->nBlasNodes < 65536u && T.tnodes.size() / 4 < 65536u;
        if (small && sb != c->stagedBlas.end() && sb->second.tri0 == L0->idxOffset) {
            S.sbNode0 = sb->first; S.sbRec = sb->second.rec; S.sbRecN = sb->second.recN;
            S.sbTri0 = sb->second.tri0; S.sbTriN = sb->second.triN;
        }
    }
}

int buildInstanceTables(surf_ctx* c, const surf_gpu_instance* instances, uint32_t n, const uint32_t* tlasIdx,
                        const surf_bvh_node* tlasNodes, uint32_t nTlas, const surf_light* lights, uint32_t nLights, InstanceTables& T) {
    auto affine = [](const float* m) { return m[3] == 0.0f && m[7] == 0.0f && m[11] == 0.0f && m[15] == 1.0f; };
    T.inst.resize(n);
    T.tinst.resize(n);
    for (uint32_t i = 0; i < n; ++i) {
        const surf_gpu_instance& g = instances[i];
        const auto root = c->blasRoots.find(std::make_tuple(g.bvh_node_offset, g.bvh_idx_offset, g.tri_offset));
        if (root == c->blasRoots.end() || g.material_offset >= c->nMaterials)
            return fail(c, SURF_ERR_INVALID, "instance " + std::to_string(i) + ": offsets do not name an uploaded BLAS/material");
        DevInstance& D = T.inst[i];
        std::memcpy(D.Minv, g.inv_transform, sizeof D.Minv);
        std::memcpy(D.M, g.transform, sizeof D.M);
        D.triOffset = g.tri_offset; D.idxOffset = g.bvh_idx_offset; D.nodeOffset = g.bvh_node_offset; D.material = g.material_offset;
        D.area = g.area;
        /* row 3 of a column-major matrix: elements 3, 7, 11, 15 */
        D.affineInv = affine(g.inv_transform) ? 1u : 0u;
        D.affine = affine(g.transform) ? 1u : 0u;
        const float* m = D.Minv;
        TraceInst& R = T.tinst[i];
        R.m0 = make_float4(m[0], m[4], m[8], m[12]);
        R.m1 = make_float4(m[1], m[5], m[9], m[13]);
        R.m2 = make_float4(m[2], m[6], m[10], m[14]);
        R.m3 = make_float4(m[3], m[7], m[11], m[15]);
        R.meta = make_uint4(D.nodeOffset, D.idxOffset, D.affineInv, i);
        R.r0 = root->second[0]; R.r1 = root->second[1]; R.r2 = root->second[2]; R.r3 = root->second[3];
        /* conservative world box: the triangle bounds' corners mapped to world
         * space by the inverse of the M^-1 the traversal applies (inverted in
         * double, so the box matches the object-space rays whatever M says),
         * padded by 1e-4 of the box's coordinate magnitude times the matrix's
         * condition number (~1000x the float rounding of the ray transform,
         * slab terms and triangle test); not usable (never culls) for a
         * projective or singular M^-1 or non-finite bounds */
        R.wlo = make_float4(0, 0, 0, 0);
        R.whi = make_float4(0, 0, 0, 0);
        const auto bb = c->blasBounds.find(g.tri_offset);
        double A[3][3], t[3], B[3][3];      /* M^-1 = [A t; 0 1] (column-major input), B = A^-1 */
        for (int r = 0; r < 3; ++r) {
            for (int q = 0; q < 3; ++q) A[r][q] = (double)g.inv_transform[4 * q + r];
            t[r] = (double)g.inv_transform[12 + r];
        }
        const double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) - A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                           A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
        if (bb != c->blasBounds.end() && D.affineInv && std::isfinite(det) && det != 0.0) {
            B[0][0] = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det; B[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
            B[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det; B[1][0] = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
            B[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det; B[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
            B[2][0] = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det; B[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
            B[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
            double na = 0.0, nb = 0.0;
            for (int r = 0; r < 3; ++r)
                for (int q = 0; q < 3; ++q) { na += A[r][q] * A[r][q]; nb += B[r][q] * B[r][q]; }
            const double cond = std::sqrt(na * nb);
            double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
            for (int corner = 0; corner < 8; ++corner) {
                const double p[3] = {bb->second[(corner & 1) ? 3 : 0] - t[0], bb->second[(corner & 2) ? 4 : 1] - t[1],
                                     bb->second[(corner & 4) ? 5 : 2] - t[2]};
                for (int r = 0; r < 3; ++r) {
                    const double w = B[r][0] * p[0] + B[r][1] * p[1] + B[r][2] * p[2];
                    lo[r] = std::min(lo[r], w); hi[r] = std::max(hi[r], w);
                }
            }
            double mag = 0.0;
            for (int r = 0; r < 3; ++r) mag = std::max({mag, std::fabs(lo[r]), std::fabs(hi[r]), hi[r] - lo[r]});
            const double pad = 1e-4 * mag * std::max(1.0, cond) + 1e-6;
            bool ok = std::isfinite(mag) && mag < 1e30;
            float flo[3], fhi[3];
            for (int r = 0; r < 3; ++r) {
                flo[r] = (float)(lo[r] - pad); fhi[r] = (float)(hi[r] + pad);
                ok = ok && std::isfinite(flo[r]) && std::isfinite(fhi[r]);
            }
            if (ok) {
                R.wlo = make_float4(flo[0], flo[1], flo[2], 1.0f);
                R.whi = make_float4(fhi[0], fhi[1], fhi[2], 0.0f);
            }
        }
    }
    T.tnodes.assign((size_t)nTlas * 4, make_float4(0, 0, 0, 0));
    std::vector<uint8_t> tseen(n, 0);
    TreeWalk tw = walkTree(tlasNodes, nTlas, 0, n, 0, T.tnodes, tseen);
    if (!tw.ok) return fail(c, SURF_ERR_INVALID, "TLAS: " + tw.why);
    T.tlasDepth = tw.depth;
    T.tidx.assign(tlasIdx, tlasIdx + n);
    for (uint32_t v : T.tidx) if (v >= n) return fail(c, SURF_ERR_INVALID, "TLAS index out of range");
    T.tlasLeafCount = tlasNodes[0].count;        /* root leaf: wave-uniform instance loop */
    if (T.tlasLeafCount && tlasNodes[0].left_first != 0) T.tlasLeafCount = 0;   /* general path unless indices start at 0 */
    /* ray-order membership key: the (at most 3) instances of a single-leaf
     * TLAS with the largest BLASes (>= 64 triangles) and a usable world box */
    if (T.tlasLeafCount) {
        std::vector<std::pair<uint32_t, uint32_t>> big;     /* (triangles, instance) */
        for (uint32_t i = 0; i < n; ++i) {
            const auto it = c->blasSlots.find(instances[i].tri_offset);
            const uint32_t tris = it == c->blasSlots.end() ? 0u : it->second;
            if (tris >= 64 && T.tinst[i].wlo.w != 0.0f) big.push_back({tris, i});
        }
        std::stable_sort(big.begin(), big.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
        for (size_t h = 0; h < big.size() && h < 3; ++h) {
            T.hvLo[h] = T.tinst[big[h].second].wlo;
            T.hvHi[h] = T.tinst[big[h].second].whi;
            T.hvInst[h] = big[h].second;
            T.nHeavy = (uint32_t)h + 1;
        }
    }
    T.lights.resize(nLights);
    for (uint32_t l = 0; l < nLights; ++l) {
        const surf_light& L = lights[l];
        if (L.light_instance_idx >= n || L.primitive_count == 0 ||
            (uint64_t)instances[L.light_instance_idx].tri_offset + L.primitive_count > c->nTriangles)
            return fail(c, SURF_ERR_INVALID, "light " + std::to_string(l) + " out of range");
        T.lights[l] = make_uint2(L.light_instance_idx, L.primitive_count);
    }
    return SURF_OK;
}

int surf_upload_scene(surf_ctx* c, const surf_scene_desc* d) {
    if (!c || !d) return SURF_ERR_INVALID;
    if (d->triangle_count == 0 || !d->triangles || !d->tri_ext || !d->blas_indices || !d->blas_nodes || !d->materials ||
        !d->instances || d->instance_count == 0 || !d->tlas_indices || !d->tlas_nodes || d->tlas_node_count == 0 ||
        !d->background || d->material_count == 0 || d->blas_node_count == 0 || d->blas_index_count == 0 ||
        (d->light_count && !d->lights))
        return fail(c, SURF_ERR_INVALID, "incomplete scene descriptor");
    /* the kernels index records with 32-bit element offsets (16 floats per node,
     * 12 per BLAS index slot, 16 per triangle record) */
    if (d->blas_node_count >= (1u << 28) || d->blas_index_count >= (1u << 28) || d->triangle_count >= (1u << 28))
        return fail(c, SURF_ERR_LIMIT, "scene larger than 2^28 BVH nodes / index slots / triangles");
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc0 = endStream(c);
    if (rc0) return rc0;
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    destroyGraph(c);
    freeList(c->sceneAllocs);
    c->hasScene = false;

    /* instances */
    std::vector<DevInstance> inst(d->instance_count);
    std::vector<int64_t> idxTri(d->blas_index_count, -1);   /* idx slot -> tri offset owner */
    std::vector<float4> nodes((size_t)d->blas_node_count * 4, make_float4(0, 0, 0, 0));
    std::vector<uint8_t> seen(d->blas_index_count, 0), walked(d->blas_node_count, 0);
    std::vector<uint32_t> owner(d->blas_node_count, kUnset);    /* BLAS node offset of every reachable node */
    uint32_t maxBlasDepth = 0;
    for (uint32_t i = 0; i < d->instance_count; ++i) {
        const surf_gpu_instance& g = d->instances[i];
        if (g.tri_offset >= d->triangle_count || g.material_offset >= d->material_count ||
            g.bvh_node_offset >= d->blas_node_count || g.bvh_idx_offset >= d->blas_index_count)
            return fail(c, SURF_ERR_INVALID, "instance " + std::to_string(i) + " offsets out of range");
        DevInstance& D = inst[i];
        std::memcpy(D.Minv, g.inv_transform, sizeof D.Minv);
        std::memcpy(D.M, g.transform, sizeof D.M);
        D.triOffset = g.tri_offset; D.idxOffset = g.bvh_idx_offset; D.nodeOffset = g.bvh_node_offset; D.material = g.material_offset;
        D.area = g.area;
        /* row 3 of a column-major matrix: elements 3, 7, 11, 15 */
        auto affine = [](const float* m) { return m[3] == 0.0f && m[7] == 0.0f && m[11] == 0.0f && m[15] == 1.0f; };
        D.affineInv = affine(g.inv_transform) ? 1u : 0u;
        D.affine = affine(g.transform) ? 1u : 0u;
        if (!walked[g.bvh_node_offset]) {
            std::vector<uint8_t> leaf(d->blas_index_count, 0);
            TreeWalk w = walkTree(d->blas_nodes, d->blas_node_count, g.bvh_node_offset, d->blas_index_count, g.bvh_idx_offset, nodes, leaf,
                                  &owner);
            if (!w.ok) return fail(c, SURF_ERR_INVALID, "instance " + std::to_string(i) + ": " + w.why);
            maxBlasDepth = std::max(maxBlasDepth, w.depth);
            walked[g.bvh_node_offset] = 1;
            for (uint32_t k = 0; k < d->blas_index_count; ++k)
                if (leaf[k]) {
                    if (idxTri[k] >= 0 && idxTri[k] != (int64_t)g.tri_offset) return fail(c, SURF_ERR_INVALID, "BLAS index range shared by two meshes");
                    idxTri[k] = g.tri_offset;
                }
        }
    }
    c->nBlasNodes = d->blas_node_count;
    /* the compact form of every small BLAS (k_connect stages the emitters' one,
     * blasAnyStaged): its interior records in DFS order from the root (record 0),
     * each child an interior record index or a leaf's kLeafTagC | count << 16 |
     * leftFirst; and the span of its triangle slots */
    std::map<uint32_t, std::vector<float4>> compact;
    std::map<uint32_t, std::array<uint32_t, 2>> compactTris;   /* node offset -> (index offset, slots) */
    for (uint32_t i = 0; i < d->instance_count; ++i) {
        const uint32_t root = d->instances[i].bvh_node_offset;
        if (compact.count(root) || d->blas_nodes[root].count != 0) continue;
        std::vector<float4> recs;
        std::vector<uint32_t> order{root};                     /* interior nodes by record index */
        uint32_t slots = 0;
        bool ok = true;
        for (size_t k = 0; k < order.size() && ok; ++k) {
            const uint32_t g = order[k];
            const float4* r = &nodes[4 * (size_t)g];
            uint32_t ref[2];
            for (int ch = 0; ch < 2; ++ch) {
                const uint32_t cg = root + f2u(r[0].w) + (uint32_t)ch;
                const surf_bvh_node& q = d->blas_nodes[cg];
                if (q.count != 0) {
                    ok = ok && q.count < 32768u && q.left_first < 65536u;
                    ref[ch] = kLeafTagC | (q.count << 16) | (q.left_first & 0xffffu);
                    slots = std::max(slots, q.left_first + q.count);
                } else {
                    ok = ok && order.size() < 32768u;
                    ref[ch] = (uint32_t)order.size();
                    order.push_back(cg);
                }
            }
            recs.push_back(make_float4(r[0].x, r[0].y, r[0].z, u2f(ref[0])));
            recs.push_back(make_float4(r[1].x, r[1].y, r[1].z, u2f(ref[1])));
            recs.push_back(make_float4(r[2].x, r[2].y, r[2].z, 0.0f));
            recs.push_back(make_float4(r[3].x, r[3].y, r[3].z, 0.0f));
            ok = ok && (recs.size() / 4) * 64 + (uint64_t)slots * 48 <= kLdsLightBlas;
        }
        if (ok) { compact[root] = std::move(recs); compactTris[root] = {d->instances[i].bvh_idx_offset, slots}; }
    }
    c->blasRoots.clear();
    for (uint32_t i = 0; i < d->instance_count; ++i) {
        const surf_gpu_instance& g = d->instances[i];
        const size_t r = 4 * (size_t)g.bvh_node_offset;
        c->blasRoots[std::make_tuple(g.bvh_node_offset, g.bvh_idx_offset, g.tri_offset)] = {nodes[r], nodes[r + 1], nodes[r + 2], nodes[r + 3]};
    }
    c->nTriangles = d->triangle_count;
    c->nMaterials = d->material_count;
    /* BVH-ordered triangles: (v0, prim), e1 = v1 - v0, e2 = v2 - v0 (mesh.cpp:25-26) */
    std::vector<float4> tris((size_t)d->blas_index_count * 3, make_float4(0, 0, 0, 0));
    for (uint32_t k = 0; k < d->blas_index_count; ++k) {
        if (idxTri[k] < 0) continue;
        const uint64_t t = (uint64_t)idxTri[k] + d->blas_indices[k];
        if (t >= d->triangle_count) return fail(c, SURF_ERR_INVALID, "BLAS index " + std::to_string(k) + " out of range");
        const surf_triangle& T = d->triangles[t];
        tris[3 * (size_t)k + 0] = make_float4(T.v0.x, T.v0.y, T.v0.z, u2f(d->blas_indices[k]));
        tris[3 * (size_t)k + 1] = make_float4(T.v1.x - T.v0.x, T.v1.y - T.v0.y, T.v1.z - T.v0.z, 0.0f);
        tris[3 * (size_t)k + 2] = make_float4(T.v2.x - T.v0.x, T.v2.y - T.v0.y, T.v2.z - T.v0.z, 0.0f);
    }
    /* object-space bounds of each BLAS's triangles as the traversal sees them
     * (v0, v0 + e1, v0 + e2 of the slot records), for the world-box cull */
    c->blasBounds.clear();
    c->blasSlots.clear();
    for (uint32_t k = 0; k < d->blas_index_count; ++k) {
        if (idxTri[k] < 0) continue;
        ++c->blasSlots[(uint32_t)idxTri[k]];
        auto it = c->blasBounds.emplace((uint32_t)idxTri[k], std::array<double, 6>{HUGE_VAL, HUGE_VAL, HUGE_VAL, -HUGE_VAL, -HUGE_VAL, -HUGE_VAL}).first;
        const float4 a = tris[3 * (size_t)k], e1 = tris[3 * (size_t)k + 1], e2 = tris[3 * (size_t)k + 2];
        const double v[3][3] = {{a.x, a.y, a.z}, {(double)a.x + e1.x, (double)a.y + e1.y, (double)a.z + e1.z},
                                {(double)a.x + e2.x, (double)a.y + e2.y, (double)a.z + e2.z}};
        for (const auto& p : v)
            for (int q = 0; q < 3; ++q) { it->second[q] = std::min(it->second[q], p[q]); it->second[3 + q] = std::max(it->second[3 + q], p[q]); }
    }
    std::vector<float4> normals((size_t)d->triangle_count * 3), verts((size_t)d->triangle_count * 4);
    for (uint32_t t = 0; t < d->triangle_count; ++t) {
        const surf_tri_extension& x = d->tri_ext[t];
        normals[3 * (size_t)t + 0] = make_float4(x.n0.x, x.n0.y, x.n0.z, 0.0f);
        normals[3 * (size_t)t + 1] = make_float4(x.n1.x, x.n1.y, x.n1.z, 0.0f);
        normals[3 * (size_t)t + 2] = make_float4(x.n2.x, x.n2.y, x.n2.z, 0.0f);
        const surf_triangle& T = d->triangles[t];
        verts[4 * (size_t)t + 0] = make_float4(T.v0.x, T.v0.y, T.v0.z, 0.0f);
        verts[4 * (size_t)t + 1] = make_float4(T.v1.x, T.v1.y, T.v1.z, 0.0f);
        verts[4 * (size_t)t + 2] = make_float4(T.v2.x, T.v2.y, T.v2.z, 0.0f);
        verts[4 * (size_t)t + 3] = make_float4(T.centroid.x, T.centroid.y, T.centroid.z, 0.0f);
    }
    InstanceTables IT;
    int rcT = buildInstanceTables(c, d->instances, d->instance_count, d->tlas_indices, d->tlas_nodes, d->tlas_node_count,
                                  d->lights, d->light_count, IT);
    if (rcT) return rcT;
    std::vector<DevMaterial> mats(d->material_count);
    std::memcpy(mats.data(), d->materials, d->material_count * sizeof(DevMaterial));

    const uint32_t depth = IT.tlasDepth + maxBlasDepth + 1;
    if (depth > kMaxStack) return fail(c, SURF_ERR_LIMIT, "BVH too deep for the LDS traversal stack (" + std::to_string(depth) + " entries)");

    DevScene S{};
    int rc;
    if ((rc = upload(c, nodes, &S.nodes))) return rc;
    /* two-level records for the wave walk (blasWalk2): W(g) = the records of g
     * and of its two children, each in the lanes-as-planes order (lane l of a
     * row = dword planeDword(l) of the 64-B record), 48 floats; a leaf's W holds
     * its own record.  192-B offsets are 32-bit buffer offsets: at most 22.3 M nodes. */
    const bool walk2 = !(std::getenv("SURF_WALK2") && std::getenv("SURF_WALK2")[0] == '0');   /* A/B: 0 = one-level walk (read per upload) */
    if (walk2 && (uint64_t)d->blas_node_count * 192u < (1ull << 32)) {
        std::vector<float> W((size_t)d->blas_node_count * 48, 0.0f);
        /* lanes 14 / 15 of a row (unused by the wave walk): the row node's two
         * children as packed leaf references for the lane walk (blasTraceW):
         * kLeafTag | count << 24 | leftFirst, 0 when not a leaf or too large */
        auto packLeaf = [&](uint64_t m) -> uint32_t {
            const surf_bvh_node& q = d->blas_nodes[m];
            return (q.count != 0 && q.count < 128u && q.left_first < (1u << 24)) ? (kLeafTag | (q.count << 24) | q.left_first) : 0u;
        };
        auto putRec = [&](size_t g, size_t row, uint64_t src) {
            const float* r = reinterpret_cast<const float*>(&nodes[4 * src]);
            for (uint32_t l = 0; l < 14; ++l) {
                const uint32_t dw = l < 12u ? (l / 6u) * 8u + (l & 1u) * 4u + ((l % 6u) >> 1) : (l == 12u ? 3u : 7u);
                W[48 * g + 16 * row + l] = r[dw];
            }
            const surf_bvh_node& q = d->blas_nodes[src];
            if (q.count == 0 && owner[src] != kUnset) {
                W[48 * g + 16 * row + 14] = u2f(packLeaf((uint64_t)owner[src] + q.left_first));
                W[48 * g + 16 * row + 15] = u2f(packLeaf((uint64_t)owner[src] + q.left_first + 1));
            }
        };
        /* a leaf's W holds its own record in row 0 and, for <= kLeafInW
         * triangles, the triangles themselves (row j: lanes 0..2 v0, 3..5 e1,
         * 6..8 e2, 9 prim -- the BVH-ordered records of its index slots), so the
         * wave walk tests them from the record its visit loaded (leafWaveW) */
        std::map<uint32_t, uint32_t> idxOfNode;                      /* BLAS node offset -> index offset */
        for (uint32_t i = 0; i < d->instance_count; ++i) idxOfNode[d->instances[i].bvh_node_offset] = d->instances[i].bvh_idx_offset;
        for (uint32_t g = 0; g < d->blas_node_count; ++g) {
            if (owner[g] == kUnset) continue;
            putRec(g, 0, g);
            const surf_bvh_node& n = d->blas_nodes[g];
            if (n.count == 0) {
                putRec(g, 1, (uint64_t)owner[g] + n.left_first);
                putRec(g, 2, (uint64_t)owner[g] + n.left_first + 1);
            } else if (n.count <= kLeafInW) {
                const uint64_t slot0 = (uint64_t)idxOfNode[owner[g]] + n.left_first;
                for (uint32_t j = 0; j < n.count; ++j) {
                    const float4* t = &tris[3 * (slot0 + j)];
                    float* w = &W[48 * (size_t)g + 16 * j];
                    w[0] = t[0].x; w[1] = t[0].y; w[2] = t[0].z;
                    w[3] = t[1].x; w[4] = t[1].y; w[5] = t[1].z;
                    w[6] = t[2].x; w[7] = t[2].y; w[8] = t[2].z;
                    w[9] = t[0].w;
                }
            }
        }
        const float* dW = nullptr;
        if ((rc = upload(c, W, &dW))) return rc;
        S.wnodes = dW;
        S.nWnodes = d->blas_node_count;
        /* the lane traversal walks them too when the BVH cannot stay in the
         * caches (nodes + triangles past the 256 MB of MALL): one DRAM round
         * trip per two levels instead of one per level (SURF_LANEW=0|1: A/B) */
        const uint64_t bvhBytes = (uint64_t)d->blas_node_count * 64u + (uint64_t)d->blas_index_count * 48u;
        S.laneW = bvhBytes > (256ull << 20) ? 1u : 0u;
        if (const char* e = std::getenv("SURF_LANEW")) S.laneW = e[0] == '1' ? 1u : 0u;
    }
    if ((rc = upload(c, tris, &S.tris))) return rc;
    if ((rc = upload(c, normals, &S.normals))) return rc;
    if ((rc = upload(c, verts, &S.verts))) return rc;
    if ((rc = upload(c, IT.tnodes, &S.tlasNodes))) return rc;
    if ((rc = upload(c, IT.tidx, &S.tlasIdx))) return rc;
    if ((rc = upload(c, IT.inst, &S.inst))) return rc;
    if ((rc = upload(c, IT.tinst, &S.tinst))) return rc;
    if ((rc = upload(c, mats, &S.mats))) return rc;
    if ((rc = upload(c, IT.lights, &S.lights))) return rc;
    S.nLights = d->light_count;
    S.nInst = d->instance_count;
    S.nMats = d->material_count;
    S.nodes4G = d->blas_node_count < (1u << 26) ? 1u : 0u;
    S.finiteBoxes = 1u;
    for (const float4& q : nodes)
        if (!(std::fabs(q.x) <= FLT_MAX && std::fabs(q.y) <= FLT_MAX && std::fabs(q.z) <= FLT_MAX)) { S.finiteBoxes = 0u; break; }
    S.tlasLeafCount = IT.tlasLeafCount;
    c->stagedBlas.clear();
    for (const auto& kv : compact) {
        const float4* dR = nullptr;
        if ((rc = upload(c, kv.second, &dR))) return rc;
        c->stagedBlas[kv.first] = surf_ctx::StagedBlas{dR, (uint32_t)(kv.second.size() / 4), compactTris[kv.first][0],
                                                        compactTris[kv.first][1]};
    }
    setKeys(c, S, IT);
    const surf_background& bg = *d->background;
    S.bgType = bg.type;
    S.bgColor[0] = bg.color.x; S.bgColor[1] = bg.color.y; S.bgColor[2] = bg.color.z;
    S.bgA[0] = bg.gradient_a.x; S.bgA[1] = bg.gradient_a.y; S.bgA[2] = bg.gradient_a.z;
    S.bgB[0] = bg.gradient_b.x; S.bgB[1] = bg.gradient_b.y; S.bgB[2] = bg.gradient_b.z;
    {
        /* ray-order cells (a sort key only: any value is correct, a stale box after refits too) */
        const surf_bvh_node& root = d->tlas_nodes[0];
        const float lo[3] = {root.bb_min.x, root.bb_min.y, root.bb_min.z}, hi[3] = {root.bb_max.x, root.bb_max.y, root.bb_max.z};
        for (int a = 0; a < 3; ++a) {
            const float ext = hi[a] - lo[a];
            const bool ok = std::isfinite(lo[a]) && std::isfinite(ext) && ext > 0.0f;
            S.cellLo[a] = ok ? lo[a] : 0.0f;
            S.cellScale[a] = ok ? 2.0f / ext : 0.0f;
        }
    }
    c->S = S;
    c->ldsTables = d->instance_count <= kLdsInst && d->instance_count <= kLdsTraceInst && d->material_count <= kLdsMats &&
                   d->light_count <= kLdsLights;
    c->stackDepth = depth;
    c->nInstances = d->instance_count;
    c->nLightsUp = d->light_count;
    c->tlasNodeCount = d->tlas_node_count;
    c->maxBlasDepth = maxBlasDepth;
    c->hasScene = true;
    return SURF_OK;
}

int surf_update_instances(surf_ctx* c, const surf_gpu_instance* instances, uint32_t n, const uint32_t* tlasIdx,
                          const surf_bvh_node* tlasNodes, uint32_t nTlas, const surf_light* lights, uint32_t nLights) {
    if (!c || !instances || !tlasIdx || !tlasNodes || (nLights && !lights)) return SURF_ERR_INVALID;
    if (!c->hasScene) return fail(c, SURF_ERR_NO_SCENE, "no scene uploaded");
    if (n != c->nInstances || nTlas != c->tlasNodeCount || nLights != c->nLightsUp)
        return fail(c, SURF_ERR_INVALID, "instance/TLAS/light counts differ from the uploaded scene: use surf_upload_scene");
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc = endStream(c);            /* in-flight paths belong to the old transforms */
    if (rc) return rc;
    InstanceTables IT;
    if ((rc = buildInstanceTables(c, instances, n, tlasIdx, tlasNodes, nTlas, lights, nLights, IT))) return rc;
    const uint32_t depth = IT.tlasDepth + c->maxBlasDepth + 1;
    if (depth > kMaxStack) return fail(c, SURF_ERR_LIMIT, "BVH too deep for the LDS traversal stack (" + std::to_string(depth) + " entries)");
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    auto put = [&](const void* dst, const void* src, size_t bytes) {
        return hipMemcpy(const_cast<void*>(dst), src, bytes, hipMemcpyHostToDevice);
    };
    SURF_CHECK(c, put(c->S.inst, IT.inst.data(), IT.inst.size() * sizeof(DevInstance)));
    SURF_CHECK(c, put(c->S.tinst, IT.tinst.data(), IT.tinst.size() * sizeof(TraceInst)));
    SURF_CHECK(c, put(c->S.tlasNodes, IT.tnodes.data(), IT.tnodes.size() * sizeof(float4)));
    SURF_CHECK(c, put(c->S.tlasIdx, IT.tidx.data(), IT.tidx.size() * sizeof(uint32_t)));
    if (nLights) SURF_CHECK(c, put(c->S.lights, IT.lights.data(), IT.lights.size() * sizeof(uint2)));
    c->S.tlasLeafCount = IT.tlasLeafCount;
    setKeys(c, c->S, IT);
    c->stackDepth = std::max(c->stackDepth, depth);
    destroyGraph(c);                  /* kernel arguments carry the scene descriptor */
    return SURF_OK;
}

int surf_set_camera(surf_ctx* c, const surf_camera_ubo* u) {
    if (!c || !u) return SURF_ERR_INVALID;
    if (c->hasCamera && std::memcmp(u, &c->camUbo, sizeof *u) == 0) return SURF_OK;   /* unchanged: keep the stream */
    int rc0 = endStream(c);
    if (rc0) return rc0;
    if (!(u->resolution[0] > 0.0f) || !(u->resolution[1] > 0.0f)) return fail(c, SURF_ERR_INVALID, "camera resolution must be positive");
    DevCamera k{};
    const float pos[3] = {u->position.x, u->position.y, u->position.z};
    std::memcpy(k.pos, pos, sizeof pos);
    k.firstPixel[0] = u->first_pixel.x; k.firstPixel[1] = u->first_pixel.y; k.firstPixel[2] = u->first_pixel.z;
    k.uVec[0] = u->u_vector.x; k.uVec[1] = u->u_vector.y; k.uVec[2] = u->u_vector.z;
    k.vVec[0] = u->v_vector.x; k.vVec[1] = u->v_vector.y; k.vVec[2] = u->v_vector.z;
    k.invW = 1.0f / u->resolution[0];
    k.invH = 1.0f / u->resolution[1];
    k.defocus = (u->defocus_angle == 0.0f) ? 0u : 1u;
    /* sampleDefocusDisk constants (camera.h:73-75), computed once on the host */
    const V3 up = mk3(u->up.x, u->up.y, u->up.z), fwd = mk3(u->fwd.x, u->fwd.y, u->fwd.z);
    const V3 right = normalize(cross(up, fwd));
    const float deg = u->defocus_angle / 2.0f;
    const float radius = u->focal_length * tanf((deg * 3.14159265358979323846264f) * 0.005555555555555f);
    const V3 du = scl(right, radius), dv = scl(lscl(-1.0f, up), radius);
    k.diskU[0] = du.x; k.diskU[1] = du.y; k.diskU[2] = du.z;
    k.diskV[0] = dv.x; k.diskV[1] = dv.y; k.diskV[2] = dv.z;
    c->cam = k;
    c->permValid = false;
    c->camUbo = *u;
    c->hasCamera = true;
    destroyGraph(c);     /* camera is a kernel argument of the captured graph */
    return SURF_OK;
}

int surf_render(surf_ctx* c, uint32_t frames, uint32_t firstSample, uint32_t maxSeg, uint32_t spp) {
    if (!c) return SURF_ERR_INVALID;
    if (spp == 0 || spp > 4096) return fail(c, SURF_ERR_INVALID, "samples_per_frame must be 1..4096");
    if (!c->hasScene) return fail(c, SURF_ERR_NO_SCENE, "no scene uploaded");
    if (!c->hasCamera) return fail(c, SURF_ERR_NO_SCENE, "no camera set");
    if (frames == 0) return SURF_OK;
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc = allocWavefront(c);
    if (rc) return rc;
    /* continue the open stream only for the next consecutive frames of the same kind */
    if (c->streamActive && ((uint64_t)firstSample != c->baseFrame + targetPasses(c) || maxSeg != c->streamMaxSeg || spp != c->spp))
        if ((rc = endStream(c))) return rc;
    if (!c->streamActive) {
        if ((rc = ensureWindow(c, frames, spp))) return rc;
        if ((rc = startStream(c, firstSample, maxSeg, frames, spp))) return rc;
    }
    if (!c->profiling && (rc = buildGraph(c))) return rc;         /* (re)captured if the ring moved */
    /* this call's device time: an event pair of its own (the pair two calls
     * back is read first, if that call returned with replays in flight) */
    const int tp = c->tevCur;
    if (c->tevPending[tp]) {
        SURF_CHECK(c, hipEventSynchronize(c->tev[tp][1]));
        float ms0 = 0;
        (void)hipEventElapsedTime(&ms0, c->tev[tp][0], c->tev[tp][1]);
        c->stats.ms_total += ms0;
        c->tevPending[tp] = false;
    }
    SURF_CHECK(c, hipEventRecord(c->tev[tp][0], c->stream));
    c->targetFrames += frames;
    /* A one-frame call (the drop-in loop, main.cpp:381-446) may return with up
     * to a pool's worth of its stream not yet issued: the next calls, or the
     * drain a read of the accumulator starts, issue it.  Issuing each call's
     * frame at once would run a short replay per frame on a pool a third full
     * (DESIGN 4 "Pool sizing"); with the lag the pool stays full and the
     * calls replay only as many phases as the stream retires. */
    const uint64_t lag = frames == 1 && c->loopLag ? c->capacity : 0;
    if ((rc = pump(c, false, lag))) return rc;
    SURF_CHECK(c, hipEventRecord(c->tev[tp][1], c->stream));
    if (c->snapCount) {
        /* replays still in flight (a pipelined one-frame call): timed when read */
        c->tevPending[tp] = true;
        c->tevCur ^= 1;
    } else {
        SURF_CHECK(c, hipEventSynchronize(c->tev[tp][1]));
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->tev[tp][0], c->tev[tp][1]);
        c->stats.ms_total += ms;
    }
    c->totalSamples += (uint64_t)frames * spp;
    c->stats.samples += (uint64_t)frames * spp * c->npx;
    return SURF_OK;
}

int surf_clear_accumulator(surf_ctx* c) {
    if (!c) return SURF_ERR_INVALID;
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc = endStream(c);
    if (rc) return rc;
    SURF_CHECK(c, hipMemsetAsync(c->acc, 0, (size_t)c->npx * sizeof(float4), c->stream));
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    c->totalSamples = 0;
    std::memset(&c->stats, 0, sizeof c->stats);
    std::memset(c->evBase, 0, sizeof c->evBase);
    c->segMaxBase = 0;
    c->tailFirstRays = 0;
    return SURF_OK;
}

int surf_read_accumulator(surf_ctx* c, float* out) {
    if (!c || !out) return SURF_ERR_INVALID;
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc = ensureDrained(c);
    if (rc) return rc;
    SURF_CHECK(c, hipMemcpyAsync(out, c->acc, (size_t)c->npx * sizeof(float4), hipMemcpyDeviceToHost, c->stream));
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    return SURF_OK;
}

int surf_copy_accumulator_device(surf_ctx* c, void* dst) {
    if (!c || !dst) return SURF_ERR_INVALID;
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc = ensureDrained(c);
    if (rc) return rc;
    SURF_CHECK(c, hipMemcpyAsync(dst, c->acc, (size_t)c->npx * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    return SURF_OK;
}

int surf_finalize_rgba8(surf_ctx* c, uint32_t* out) {
    if (!c || !out) return SURF_ERR_INVALID;
    if (c->totalSamples == 0) return fail(c, SURF_ERR_INVALID, "nothing rendered since the last clear");
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc = allocWavefront(c);
    if (rc) return rc;
    if ((rc = ensureDrained(c))) return rc;
    const float inv = 1.0f / (float)c->totalSamples;     /* renderer.cpp:160 */
    hipLaunchKernelGGL(k_finalize, dim3((c->npx + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream, (const float4*)c->acc,
                       c->dOutRGBA, c->npx, inv);
    SURF_CHECK(c, hipGetLastError());
    SURF_CHECK(c, hipMemcpyAsync(out, c->dOutRGBA, (size_t)c->npx * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    return SURF_OK;
}

int surf_display_rgba8(surf_ctx* c, uint32_t* out) {
    if (!c || !out) return SURF_ERR_INVALID;
    if (c->totalSamples == 0) return fail(c, SURF_ERR_INVALID, "nothing rendered since the last clear");
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc = allocWavefront(c);
    if (rc) return rc;
    if ((rc = ensureDrained(c))) return rc;
    const float inv = 1.0f / (float)c->totalSamples;
    hipLaunchKernelGGL(k_display, dim3((c->npx + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream, (const float4*)c->acc,
                       c->dOutRGBA, c->npx, inv);
    SURF_CHECK(c, hipGetLastError());
    SURF_CHECK(c, hipMemcpyAsync(out, c->dOutRGBA, (size_t)c->npx * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    return SURF_OK;
}

int surf_get_stats(surf_ctx* c, surf_stats* out) {
    if (!c || !out) return SURF_ERR_INVALID;
    int rc = ensureDrained(c);
    if (rc) return rc;
    surf_stats s = c->stats;
    unsigned long long ev[kEvents];
    unsigned long long cur[kEvents] = {};
    if (c->streamActive && c->hctr) streamEvents(*c->hctr, cur);
    for (int k = 0; k < kEvents; ++k) ev[k] = c->evBase[k] + cur[k];
    s.n_ext = ev[0]; s.n_hit = ev[1]; s.n_cont = ev[2]; s.n_shadow = ev[3]; s.n_acc = ev[4]; s.n_unocc = ev[5];
    s.tail_paths = ev[6];
    s.n_ext_wavefront = ev[8] - c->tailFirstRays;
    s.max_segments = std::max(c->segMaxBase, (c->streamActive && c->hctr) ? c->hctr->segMax : 0u);
    s.stack_depth = c->stackDepth;
    s.pool_capacity = c->capacity;
    s.frame_window = c->window;
    if (c->totalSamples) {
        /* Lumen energy, renderer.cpp:191-201: per-pixel terms on the GPU
         * (k_energy_terms), then the reference's serial sum in pixel order */
        if ((rc = allocWavefront(c))) return rc;
        const float inv = 1.0f / (float)c->totalSamples;
        float* terms = reinterpret_cast<float*>(c->dOutRGBA);          /* npx words, reused */
        hipLaunchKernelGGL(k_energy_terms, dim3((c->npx + kBlock - 1) / kBlock), dim3(kBlock), 0, c->stream,
                           (const float4*)c->acc, terms, c->npx, inv);
        SURF_CHECK(c, hipGetLastError());
        std::vector<float> h(c->npx);
        SURF_CHECK(c, hipMemcpyAsync(h.data(), terms, (size_t)c->npx * sizeof(float), hipMemcpyDeviceToHost, c->stream));
        SURF_CHECK(c, hipStreamSynchronize(c->stream));
        float e = 0.0f;
        for (size_t p = 0; p < c->npx; ++p) e = e + h[p];
        s.energy = e;
    }
    *out = s;
    return SURF_OK;
}

int surf_synchronize(surf_ctx* c) {
    if (!c) return SURF_ERR_INVALID;
    SURF_CHECK(c, hipSetDevice(c->device));
    int rc = ensureDrained(c);
    if (rc) return rc;
    SURF_CHECK(c, hipStreamSynchronize(c->stream));
    return SURF_OK;
}

int surf_trace_closest(surf_ctx* c, uint32_t n, const float* o, const float* d, float* ot, float* ou, float* ov,
                       uint32_t* oi, uint32_t* op) {
    if (!c || (n && (!o || !d || !ot || !ou || !ov || !oi || !op))) return SURF_ERR_INVALID;
    if (!c->hasScene) return fail(c, SURF_ERR_NO_SCENE, "no scene uploaded");
    if (n == 0) return SURF_OK;
    if (c->traceMode == 1 && !waveEligible(c))
        return fail(c, SURF_ERR_INVALID, "scene no longer fits the selected cooperative traversal");
    SURF_CHECK(c, hipSetDevice(c->device));
    std::vector<void*> tmp;
    float *dO, *dD; float4* dT; uint2* dI;
    int rc;
    if ((rc = devAlloc(c, tmp, &dO, 3 * (size_t)n)) || (rc = devAlloc(c, tmp, &dD, 3 * (size_t)n)) ||
        (rc = devAlloc(c, tmp, &dT, n)) || (rc = devAlloc(c, tmp, &dI, n))) { freeList(tmp); return rc; }
    (void)hipMemcpyAsync(dO, o, 12 * (size_t)n, hipMemcpyHostToDevice, c->stream);
    (void)hipMemcpyAsync(dD, d, 12 * (size_t)n, hipMemcpyHostToDevice, c->stream);
    if (c->traceMode == 1)
        hipLaunchKernelGGL(c->ldsTables ? (c->S.wnodes ? k_trace_closest_coop<true, true> : k_trace_closest_coop<true, false>)
                                        : (c->S.wnodes ? k_trace_closest_coop<false, true> : k_trace_closest_coop<false, false>),
                           dim3(n), dim3(64), coopLds(c),
                           c->stream, c->S, (const float*)dO, (const float*)dD,
                           n, dT, dI, recStackWords(c));
    else
        hipLaunchKernelGGL(c->S.laneW ? (c->ldsTables ? k_trace_closest<true, true> : k_trace_closest<false, true>)
                                      : (c->ldsTables ? k_trace_closest<true, false> : k_trace_closest<false, false>),
                           dim3((n + kBlock - 1) / kBlock), dim3(kBlock), traversalLds(c, kBlock), c->stream,
                           c->S, (const float*)dO, (const float*)dD, n, dT, dI, stackWords(c, kBlock));
    std::vector<float4> t(n);
    std::vector<uint2> ip(n);
    (void)hipMemcpyAsync(t.data(), dT, 16 * (size_t)n, hipMemcpyDeviceToHost, c->stream);
    (void)hipMemcpyAsync(ip.data(), dI, 8 * (size_t)n, hipMemcpyDeviceToHost, c->stream);
    hipError_t e = hipStreamSynchronize(c->stream);
    freeList(tmp);
    if (e != hipSuccess) return fail(c, SURF_ERR_HIP, std::string("trace_closest: ") + hipGetErrorString(e));
    for (uint32_t i = 0; i < n; ++i) { ot[i] = t[i].x; ou[i] = t[i].y; ov[i] = t[i].z; oi[i] = ip[i].x; op[i] = ip[i].y; }
    return SURF_OK;
}

int surf_trace_any(surf_ctx* c, uint32_t n, const float* o, const float* d, const float* tm, uint8_t* occ) {
    if (!c || (n && (!o || !d || !tm || !occ))) return SURF_ERR_INVALID;
    if (!c->hasScene) return fail(c, SURF_ERR_NO_SCENE, "no scene uploaded");
    if (n == 0) return SURF_OK;
    if (c->traceMode == 1 && !waveEligible(c))
        return fail(c, SURF_ERR_INVALID, "scene no longer fits the selected cooperative traversal");
    SURF_CHECK(c, hipSetDevice(c->device));
    std::vector<void*> tmp;
    float *dO, *dD, *dM; uint8_t* dR;
    int rc;
    if ((rc = devAlloc(c, tmp, &dO, 3 * (size_t)n)) || (rc = devAlloc(c, tmp, &dD, 3 * (size_t)n)) ||
        (rc = devAlloc(c, tmp, &dM, n)) || (rc = devAlloc(c, tmp, &dR, n))) { freeList(tmp); return rc; }
    (void)hipMemcpyAsync(dO, o, 12 * (size_t)n, hipMemcpyHostToDevice, c->stream);
    (void)hipMemcpyAsync(dD, d, 12 * (size_t)n, hipMemcpyHostToDevice, c->stream);
    (void)hipMemcpyAsync(dM, tm, 4 * (size_t)n, hipMemcpyHostToDevice, c->stream);
    if (c->traceMode == 1)
        hipLaunchKernelGGL(c->ldsTables ? (c->S.wnodes ? k_trace_any_coop<true, true> : k_trace_any_coop<true, false>)
                                        : (c->S.wnodes ? k_trace_any_coop<false, true> : k_trace_any_coop<false, false>),
                           dim3(n), dim3(64), coopLds(c), c->stream,
                           c->S, (const float*)dO, (const float*)dD,
                           (const float*)dM, n, dR, recStackWords(c));
    else
        hipLaunchKernelGGL(c->S.laneW ? (c->ldsTables ? k_trace_any<true, true> : k_trace_any<false, true>)
                                      : (c->ldsTables ? k_trace_any<true, false> : k_trace_any<false, false>),
                           dim3((n + kBlock - 1) / kBlock), dim3(kBlock), traversalLds(c, kBlock), c->stream,
                           c->S, (const float*)dO, (const float*)dD, (const float*)dM, n, dR, stackWords(c, kBlock));
    (void)hipMemcpyAsync(occ, dR, n, hipMemcpyDeviceToHost, c->stream);
    hipError_t e = hipStreamSynchronize(c->stream);
    freeList(tmp);
    if (e != hipSuccess) return fail(c, SURF_ERR_HIP, std::string("trace_any: ") + hipGetErrorString(e));
    return SURF_OK;
}

int surf_debug_lane_resumed(surf_ctx* c, uint64_t* rays) {
    if (!c || !rays) return SURF_ERR_INVALID;
    int rc = ensureDrained(c);
    if (rc) return rc;
    unsigned long long cur[kEvents] = {};
    if (c->streamActive && c->hctr) streamEvents(*c->hctr, cur);
    *rays = c->evBase[9] + cur[9];
    return SURF_OK;
}

int surf_debug_connect_staging(surf_ctx* c, uint32_t* records, uint32_t* triangles) {
    if (!c || !records || !triangles) return SURF_ERR_INVALID;
    *records = c->connectStaged ? c->S.sbRecN : 0u;
    *triangles = c->connectStaged ? c->S.sbTriN : 0u;
    return SURF_OK;
}

int surf_debug_segment_cycles(surf_ctx* c, const float* path12, uint32_t reps, uint64_t* cycles15) {
    if (!c || !path12 || !cycles15 || reps == 0) return SURF_ERR_INVALID;
    if (!c->hasScene) return fail(c, SURF_ERR_NO_SCENE, "no scene uploaded");
    if (!waveEligible(c)) return fail(c, SURF_ERR_INVALID, "scene does not fit the one-ray-per-wave traversal");
    SURF_CHECK(c, hipSetDevice(c->device));
    unsigned long long* d = nullptr;
    SURF_CHECK(c, hipMalloc(&d, 16 * sizeof(unsigned long long)));
    const float4 o4 = make_float4(path12[0], path12[1], path12[2], path12[3]);
    const float4 d4 = make_float4(path12[4], path12[5], path12[6], path12[7]);
    const float4 T4 = make_float4(path12[8], path12[9], path12[10], path12[11]);
    const bool w2 = c->S.wnodes != nullptr;
    hipLaunchKernelGGL(c->ldsTables ? (w2 ? k_segment_cycles<true, true> : k_segment_cycles<true, false>)
                                    : (w2 ? k_segment_cycles<false, true> : k_segment_cycles<false, false>),
                       dim3(1), dim3(64), coopTailLds(c), c->stream, c->S, o4, d4, T4, reps, d, recStackWords(c));
    hipError_t e = hipMemcpyAsync(cycles15, d, 15 * sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(c, SURF_ERR_HIP, std::string("segment cycles: ") + hipGetErrorString(e));
    return SURF_OK;
}

int surf_pack_rgba8(const float* acc, uint32_t n, float inv, int display, uint32_t* out) {
    if ((n && (!acc || !out))) return fail(nullptr, SURF_ERR_INVALID, "bad arguments");
    for (uint32_t p = 0; p < n; ++p) {
        uint32_t w = 0;
        for (int k = 0; k < 4; ++k) {
            const uint32_t c8 = packChannel((acc[4 * (size_t)p + k] * inv) * 255.0f);
            w |= (display ? displayChannel(c8) : c8) << (8 * k);
        }
        out[p] = w;
    }
    return SURF_OK;
}

/* Host restatements of the glibc kernels' libm, for CPU tests (same source as the device). */
float surf_ref_sinf(float x) { return surfdev::gSinf(x); }
float surf_ref_cosf(float x) { return surfdev::gCosf(x); }
float surf_ref_expf(float x) { return surfdev::gExpf(x); }

}  // extern "C"
