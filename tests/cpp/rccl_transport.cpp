// rccl_transport.cpp — the scene shards' RCCL transport (include/NFGPUSceneShard.hpp RcclTransport,
// noahgameframe_amd/host/NFGPUShardRccl.cpp) run on the GPU at world size 1: the ticket all-gather
// (the count and the first words in one round, the rest in a second when a list is longer) and the rows' grouped ncclSend / ncclRecv to the rank itself, on the
// world's stream, device to device.  More ranks need more GPUs (the driver's 8-GPU run); this
// checks the calls, buffers and stream handling one GPU can.
// usage: rccl_transport        prints one JSON line; exit 0 when every check holds
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "NFGPUSceneShard.hpp"
#include "nfgpu.h"

using namespace nfgpu;

int main() {
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 2;
    RcclTransport t(RcclTransport::NewUniqueId(), 0, 1, (void*)s);
    int fails = 0;
    // tickets: an empty frame, then 11-word rows (kTicketWords) of three tickets
    std::vector<int64_t> all;
    fails += t.AllGather({}, all) != NFK_OK || !all.empty();
    std::vector<int64_t> mine(3 * kTicketWords);
    for (size_t i = 0; i < mine.size(); i++) mine[i] = (int64_t)(i * 7919 + 13) - 1000;
    fails += t.AllGather(mine, all) != NFK_OK || all != mine;  // (33 words: past the first round's 16)
    // the first round grows with the largest list: these fit it, then a longer one takes two rounds again
    fails += t.AllGather(mine, all) != NFK_OK || all != mine;
    fails += t.AllGather({5}, all) != NFK_OK || all != std::vector<int64_t>{5};
    std::vector<int64_t> big(300 * kTicketWords);
    for (size_t i = 0; i < big.size(); i++) big[i] = (int64_t)(i * 104729 + 7);
    fails += t.AllGather(big, all) != NFK_OK || all != big;
    fails += t.AllGather(big, all) != NFK_OK || all != big;
    // rows: 4096 words to the rank itself through RCCL, on the stream
    const size_t n = 4096;
    std::vector<uint64_t> h(n), back(n, 0);
    for (size_t i = 0; i < n; i++) h[i] = 0x9E3779B97F4A7C15ull * (i + 1);
    uint64_t *ds = nullptr, *dr = nullptr;
    if (hipMalloc(&ds, n * 8) != hipSuccess || hipMalloc(&dr, n * 8) != hipSuccess) return 2;
    if (hipMemcpy(ds, h.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess) return 2;
    fails += t.AllToAllV(ds, {n}, dr, {n}, (void*)s) != NFK_OK;
    if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(back.data(), dr, n * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    fails += back != h;
    // a frame that moves nothing
    fails += t.AllToAllV(ds, {0}, dr, {0}, (void*)s) != NFK_OK;
    fails += hipStreamSynchronize(s) != hipSuccess;
    printf("{\"rccl_transport_world_size\": 1, \"ticket_words\": %zu, \"row_words\": %zu, \"fails\": %d}\n", all.size(), n,
           fails);
    (void)hipFree(ds);
    (void)hipFree(dr);
    return fails ? 1 : 0;
}
