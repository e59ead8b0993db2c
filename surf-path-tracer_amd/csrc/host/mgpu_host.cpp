/*
 * mgpu_host.cpp -- libsurf_mgpu.so (include/surf_mgpu.h): the one collective of
 * the multi-GPU render, SURVEY.md 8e.  Row shards render independently on
 * their own devices; the float accumulators go to rank 0 with one RCCL
 * ncclGather (rccl.h:745) over xGMI -- every rank sends max-rows x width x 4
 * floats (its rows, padded to the largest shard), so the root receives
 * shard_count equal slabs -- and rank 0 un-permutes the rows into the frame.
 * Volume at C4 (1920x1080, 8 shards): 4.1 MB per rank, 33 MB in all, a few
 * tens of microseconds of xGMI against seconds of rendering: latency-bound,
 * so one flat gather, no ring or tree tuning.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "surf_mgpu.h"

struct surf_mgpu {
    surf_ctx* shard = nullptr;
    int device = 0;
    uint32_t width = 0, height = 0, index = 0, count = 1, rowBlock = 0;
    uint32_t rows = 0, maxRows = 0;      /* this shard's rows; the largest shard's */
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    float* dSend = nullptr;              /* maxRows x width x 4 */
    float* dRecv = nullptr;              /* rank 0: count x maxRows x width x 4 */
};

namespace {

std::mutex gMutex;
std::string gError;

int fail(int code, const std::string& msg) {
    std::lock_guard<std::mutex> l(gMutex);
    gError = msg;
    return code;
}

int rcclFail(const char* what, ncclResult_t r) { return fail(SURF_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r)); }
int hipFail(const char* what, hipError_t e) { return fail(SURF_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e)); }

int shardRowCount(uint32_t height, uint32_t k, uint32_t shards, uint32_t block, uint32_t* n) {
    return surf_shard_row_list(height, k, shards, block, nullptr, n);
}

/* Geometry and buffers of one rank (its communicator is set by the caller). */
int setupRank(surf_ctx* shard, uint32_t width, uint32_t height, uint32_t index, uint32_t count, uint32_t rowBlock,
              surf_mgpu** out) {
    if (!shard || !out || count == 0 || index >= count || width == 0 || height == 0) return fail(SURF_ERR_INVALID, "bad arguments");
    auto* m = new surf_mgpu();
    m->shard = shard;
    m->width = width; m->height = height; m->index = index; m->count = count; m->rowBlock = rowBlock;
    int rc = SURF_OK;
    uint32_t mine = 0;
    if ((rc = surf_shard_rows(shard, nullptr, &mine))) { delete m; return rc; }
    for (uint32_t k = 0; k < count; ++k) {
        uint32_t n = 0;
        if ((rc = shardRowCount(height, k, count, rowBlock, &n))) { delete m; return rc; }
        if (k == index && n != mine) { delete m; return fail(SURF_ERR_INVALID, "shard context does not own shard " + std::to_string(index) + "'s rows"); }
        m->maxRows = std::max(m->maxRows, n);
    }
    m->rows = mine;
    /* the shard's own device, not the calling thread's current one: a single
     * thread sets up every rank of surf_mgpu_create_all */
    if ((rc = surf_get_device(shard, &m->device))) { delete m; return rc; }
    hipError_t e = hipSetDevice(m->device);
    const size_t slab = (size_t)m->maxRows * width * 4;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&m->dSend, slab * sizeof(float));
    if (e == hipSuccess) e = hipMemset(m->dSend, 0, slab * sizeof(float));
    if (e == hipSuccess && index == 0) e = hipMalloc(&m->dRecv, slab * count * sizeof(float));
    if (e != hipSuccess) { surf_mgpu_destroy(m); return hipFail("gather buffers", e); }
    *out = m;
    return SURF_OK;
}

/* The shard's accumulator into the send slab (drains its stream). */
int stage(surf_mgpu* m) {
    if (hipSetDevice(m->device) != hipSuccess) return fail(SURF_ERR_HIP, "hipSetDevice");
    return surf_copy_accumulator_device(m->shard, m->dSend);
}

/* Every rank waits for its gather before returning, the root too when it
 * passes no frame: the next gather's stage() rewrites dSend through the shard's
 * stream, which does not order against m->stream. */
int finishRoot(surf_mgpu* root, float* frame) {
    hipError_t e = hipSetDevice(root->device);
    if (e == hipSuccess) e = hipStreamSynchronize(root->stream);
    if (e != hipSuccess) return hipFail("gather", e);
    if (!frame) return SURF_OK;
    std::vector<float> gathered((size_t)root->count * root->maxRows * root->width * 4);
    if (e == hipSuccess)
        e = hipMemcpy(gathered.data(), root->dRecv, gathered.size() * sizeof(float), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hipFail("gather readback", e);
    return surf_mgpu_assemble(root->width, root->height, root->count, root->rowBlock, gathered.data(), root->maxRows, frame);
}

}  // namespace

extern "C" {

const char* surf_mgpu_last_error(void) {
    std::lock_guard<std::mutex> l(gMutex);
    static thread_local std::string copy;
    copy = gError;
    return copy.c_str();
}

int surf_mgpu_unique_id(uint8_t id[128]) {
    if (!id) return fail(SURF_ERR_INVALID, "id is NULL");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return rcclFail("ncclGetUniqueId", r);
    std::memcpy(id, &u, sizeof u);
    return SURF_OK;
}

int surf_mgpu_create(surf_ctx* shard, uint32_t width, uint32_t height, uint32_t index, uint32_t count, uint32_t rowBlock,
                     const uint8_t id[128], surf_mgpu** out) {
    if (!id || !out) return fail(SURF_ERR_INVALID, "bad arguments");
    *out = nullptr;
    surf_mgpu* m = nullptr;
    int rc = setupRank(shard, width, height, index, count, rowBlock, &m);
    if (rc) return rc;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    const ncclResult_t r = ncclCommInitRank(&m->comm, (int)count, u, (int)index);
    if (r != ncclSuccess) { surf_mgpu_destroy(m); return rcclFail("ncclCommInitRank", r); }
    *out = m;
    return SURF_OK;
}

int surf_mgpu_create_all(surf_ctx* const* shards, uint32_t count, uint32_t width, uint32_t height, uint32_t rowBlock,
                         surf_mgpu** out) {
    if (!shards || !out || count == 0) return fail(SURF_ERR_INVALID, "bad arguments");
    std::vector<int> devs(count);
    for (uint32_t k = 0; k < count; ++k) {
        out[k] = nullptr;
        int rc = surf_get_device(shards[k], &devs[k]);
        if (rc) return fail(rc, "shard " + std::to_string(k) + ": no context");
        for (uint32_t j = 0; j < k; ++j)   /* one rank per GPU (RCCL refuses duplicate devices in one communicator) */
            if (devs[j] == devs[k])
                return fail(SURF_ERR_INVALID, "shards " + std::to_string(j) + " and " + std::to_string(k) + " share HIP device " +
                                                  std::to_string(devs[k]));
    }
    for (uint32_t k = 0; k < count; ++k) {
        int rc = setupRank(shards[k], width, height, k, count, rowBlock, &out[k]);
        if (rc) { for (uint32_t j = 0; j < k; ++j) { surf_mgpu_destroy(out[j]); out[j] = nullptr; } return rc; }
    }
    std::vector<ncclComm_t> comms(count);
    const ncclResult_t r = ncclCommInitAll(comms.data(), (int)count, devs.data());
    if (r != ncclSuccess) {
        for (uint32_t k = 0; k < count; ++k) { surf_mgpu_destroy(out[k]); out[k] = nullptr; }
        return rcclFail("ncclCommInitAll", r);
    }
    for (uint32_t k = 0; k < count; ++k) out[k]->comm = comms[k];
    return SURF_OK;
}

int surf_mgpu_gather(surf_mgpu* m, float* frame) {
    if (!m || !m->comm) return fail(SURF_ERR_INVALID, "rank not initialised");
    int rc = stage(m);
    if (rc) return rc;
    const size_t slab = (size_t)m->maxRows * m->width * 4;
    const ncclResult_t r = ncclGather(m->dSend, m->dRecv, slab, ncclFloat32, 0, m->comm, m->stream);
    if (r != ncclSuccess) return rcclFail("ncclGather", r);
    return finishRoot(m, m->index == 0 ? frame : nullptr);
}

int surf_mgpu_gather_all(surf_mgpu* const* ms, uint32_t count, float* frame) {
    if (!ms || count == 0) return fail(SURF_ERR_INVALID, "bad arguments");
    for (uint32_t k = 0; k < count; ++k) {
        if (!ms[k] || !ms[k]->comm || ms[k]->index != k || ms[k]->count != count) return fail(SURF_ERR_INVALID, "ranks out of order");
        int rc = stage(ms[k]);
        if (rc) return rc;
    }
    ncclResult_t r = ncclGroupStart();
    bool devOk = true;
    for (uint32_t k = 0; k < count && r == ncclSuccess; ++k) {
        /* never leave the group open: a failed device switch stops issuing, the group still ends */
        if (hipSetDevice(ms[k]->device) != hipSuccess) { devOk = false; break; }
        const size_t slab = (size_t)ms[k]->maxRows * ms[k]->width * 4;
        r = ncclGather(ms[k]->dSend, ms[k]->dRecv, slab, ncclFloat32, 0, ms[k]->comm, ms[k]->stream);
    }
    const ncclResult_t e = ncclGroupEnd();
    if (!devOk) return fail(SURF_ERR_HIP, "hipSetDevice");
    if (r != ncclSuccess) return rcclFail("ncclGather", r);
    if (e != ncclSuccess) return rcclFail("ncclGroupEnd", e);
    for (uint32_t k = 1; k < count; ++k) {
        (void)hipSetDevice(ms[k]->device);
        const hipError_t he = hipStreamSynchronize(ms[k]->stream);
        if (he != hipSuccess) return hipFail("gather", he);
    }
    return finishRoot(ms[0], frame);
}

void surf_mgpu_destroy(surf_mgpu* m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    if (m->comm) (void)ncclCommDestroy(m->comm);
    if (m->dSend) (void)hipFree(m->dSend);
    if (m->dRecv) (void)hipFree(m->dRecv);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

int surf_mgpu_assemble(uint32_t width, uint32_t height, uint32_t count, uint32_t rowBlock, const float* gathered,
                       uint32_t rowsPerSlab, float* frame) {
    if (!gathered || !frame || count == 0 || width == 0) return fail(SURF_ERR_INVALID, "bad arguments");
    const size_t rowFloats = (size_t)width * 4;
    std::vector<uint32_t> rows(height);
    for (uint32_t k = 0; k < count; ++k) {
        uint32_t n = 0;
        int rc = surf_shard_row_list(height, k, count, rowBlock, rows.data(), &n);
        if (rc) return rc;
        if (n > rowsPerSlab) return fail(SURF_ERR_INVALID, "slab smaller than shard " + std::to_string(k));
        const float* slab = gathered + (size_t)k * rowsPerSlab * rowFloats;
        for (uint32_t j = 0; j < n; ++j) std::memcpy(frame + rows[j] * rowFloats, slab + j * rowFloats, rowFloats * sizeof(float));
    }
    return SURF_OK;
}

}  // extern "C"
