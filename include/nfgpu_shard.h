/* nfgpu_shard.h — C-ABI of the C++ scene shards (include/NFGPUSceneShard.hpp, libnfgpu_plugin.so) for
 * a host that is not C++ (bench.py's config[2] leg drives it through ctypes).  One shard per process
 * and GPU; every call below that says "collective" is made by every rank the same number of times.
 *
 * Replaces, across shards, the part of NFCKernelModule::SwitchScene (KM:901-951) whose target scene
 * another process owns: the entity's state row leaves its world, crosses over RCCL (xGMI) and enters
 * the owner's world with the SwitchScene property writes.
 */
#ifndef NFGPU_SHARD_H
#define NFGPU_SHARD_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* rank 0 makes the RCCL communicator's 128-byte id; the host hands it to every rank out of band */
int nfs_rccl_unique_id(uint8_t* id128);
/* a shard of `world` (an nfk world) over RCCL: rank / size as in the id's communicator (collective:
 * every rank creates its shard together); owner[s] = the rank that owns scene s (s < n_scenes);
 * pid_*: the world's SceneID / GroupID / X / Y / Z property ids (-1: absent); exchange_every: the
 * ticket all-gather runs on every that-many-th nfs_end_frame */
int nfs_create_rccl(void* world, const uint8_t* id128, int32_t rank, int32_t size, const int32_t* owner,
                    int32_t n_scenes, int32_t pid_scene, int32_t pid_group, int32_t pid_x, int32_t pid_y,
                    int32_t pid_z, int32_t exchange_every, void** shard);
void nfs_destroy(void* shard);
/* SwitchScene calls into scenes other ranks own: queued departures (SceneShard::QueueSwitch) */
int nfs_queue_switch(void* shard, int32_t n, const int64_t* guid_head, const int64_t* guid_data, const int32_t* cls,
                     const int32_t* is_player, const int32_t* scene, const int32_t* group, const float* x,
                     const float* y, const float* z);
/* collective, before a frame: the rows of the last gather's plan (SceneShard::BeginFrame);
 * n_received = the arrivals, read with nfs_received */
int nfs_begin_frame(void* shard, int64_t* n_sent, int64_t* n_received);
/* the last nfs_begin_frame's arrivals (up to cap): guid, class, player flag, scene, group */
int nfs_received(void* shard, int64_t cap, int64_t* guid_head, int64_t* guid_data, int32_t* cls, int32_t* is_player,
                 int32_t* scene, int32_t* group);
/* collective, after a frame: starts the ticket gather on an exchange frame (SceneShard::EndFrame) */
int nfs_end_frame(void* shard);
/* migrated out, migrated in, transport calls, frames */
int nfs_stats(void* shard, int64_t* out4);
/* collective: NFIRankRedisModule::GetRange(type, 0, k-1) over every shard's entities
 * (NFCRankRedisModule.cpp:109-118) with property pid as the score — each rank's top k all-gathered
 * and merged in ZREVRANGE order (SceneShard::RankTop); *n_out <= k rows */
int nfs_rank_top(void* shard, int32_t pid, int32_t k, int32_t* n_out, int64_t* guid_head, int64_t* guid_data,
                 double* score);

#ifdef __cplusplus
}
#endif
#endif
