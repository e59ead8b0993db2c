/*
 * surf_mgpu.h -- C-ABI of the multi-GPU image assembly (libsurf_mgpu.so).
 *
 * The reference renders on one Vulkan device (render_context.cpp:80-91) and has
 * no collective at all.  SURVEY.md 8e's multi-GPU design shards the frame by
 * pixel rows (surf_create_sharded: interleaved blocks of row_block rows, block
 * b on shard b % shard_count, or a contiguous split for row_block 0), runs
 * every shard's wavefront loop with no communication (a sample is a function
 * of its pixel and its sample index only), and gathers the float accumulators
 * once per frame (or per run) to the root with ONE RCCL ncclGather over xGMI
 * (rccl.h:745), followed by the row un-permute.  This library is that
 * gather for C/C++ applications built on surf_hip.h / surf/surf_host.hpp;
 * libsurf_hip.so itself does not link RCCL.
 *
 * Two ways to set it up (RCCL's own two):
 *   - one process or thread per GPU: rank 0 calls surf_mgpu_unique_id and
 *     hands the 128-byte id to every rank (MPI, a socket, a file ...); each
 *     rank calls surf_mgpu_create with its shard context (ncclCommInitRank);
 *     every rank calls surf_mgpu_gather, the root receives the frame;
 *   - one process driving every GPU: surf_mgpu_create_all over the shard
 *     contexts (ncclCommInitAll); surf_mgpu_gather_all issues the ranks'
 *     gathers as one RCCL group.
 * A gather drains each shard's sample stream first (surf_copy_accumulator_device).
 * Returns 0 or a negative surf_status (surf_hip.h); nothing aborts.
 */
#ifndef SURF_MGPU_H
#define SURF_MGPU_H

#include <stdint.h>

#include "surf_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct surf_mgpu surf_mgpu;   /* one rank: a shard context, its communicator, gather buffers */

/* ncclGetUniqueId: call on rank 0, distribute the 128 bytes to every rank. */
int surf_mgpu_unique_id(uint8_t id[128]);
/* Rank shard_index of shard_count (ncclCommInitRank on the shard's device).
 * width / height: the whole frame; row_block: the shards' row interleave. */
int surf_mgpu_create(surf_ctx* shard, uint32_t width, uint32_t height, uint32_t shard_index, uint32_t shard_count,
                     uint32_t row_block, const uint8_t id[128], surf_mgpu** out);
/* One process, every GPU: shards[k] is shard k of count (each on its own
 * device); out[k] receives rank k.  ncclCommInitAll. */
int surf_mgpu_create_all(surf_ctx* const* shards, uint32_t count, uint32_t width, uint32_t height, uint32_t row_block,
                         surf_mgpu** out);
/* Rank form: the shard's accumulator rows go to rank 0 (one ncclGather of
 * max-rows x width x 4 floats per rank, rows padded to the largest shard);
 * on rank 0 `frame` (host, height x width x 4 floats) receives the assembled
 * frame, other ranks may pass NULL. */
int surf_mgpu_gather(surf_mgpu* rank, float* frame);
/* Single-process form: every rank's gather in one RCCL group; frame as above. */
int surf_mgpu_gather_all(surf_mgpu* const* ranks, uint32_t count, float* frame);
void surf_mgpu_destroy(surf_mgpu* rank);
const char* surf_mgpu_last_error(void);

/* The root's un-permute (host): `gathered` holds shard_count slabs of
 * rows_per_slab x width x 4 floats, slab k = shard k's rows in shard order
 * (padding rows ignored); writes the height x width x 4 frame. */
int surf_mgpu_assemble(uint32_t width, uint32_t height, uint32_t shard_count, uint32_t row_block, const float* gathered,
                       uint32_t rows_per_slab, float* frame);

#ifdef __cplusplus
}
#endif

#endif /* SURF_MGPU_H */
