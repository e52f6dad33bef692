// NFGPUShardRccl.cpp — RCCL transport of the scene shards (include/NFGPUSceneShard.hpp): one rank per
// GPU, rows device to device over xGMI on the world's stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>

#include "NFGPUSceneShard.hpp"
#include "nfgpu.h"

namespace nfgpu {

RowMemory DeviceRowMemory() {
    return RowMemory{[](size_t n) {
                         void* p = nullptr;
                         if (hipMalloc(&p, n ? n : 8) != hipSuccess) throw std::runtime_error("hipMalloc (shard rows)");
                         return p;
                     },
                     [](void* p) { (void)hipFree(p); },
                     [](void* d, const void* s, size_t n) {
                         if (hipMemcpy(d, s, n, hipMemcpyDeviceToDevice) != hipSuccess)
                             throw std::runtime_error("hipMemcpy (shard rows)");
                     }};
}

static void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}

std::vector<uint8_t> RcclTransport::NewUniqueId() {
    ncclUniqueId id;
    nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return std::vector<uint8_t>((const uint8_t*)&id, (const uint8_t*)&id + sizeof id);
}

RcclTransport::RcclTransport(const std::vector<uint8_t>& unique_id, int rank, int size, void* stream)
    : stream_(stream), rank_(rank), size_(size) {
    if (unique_id.size() != sizeof(ncclUniqueId)) throw std::runtime_error("RcclTransport: bad unique id");
    ncclUniqueId id;
    memcpy(&id, unique_id.data(), sizeof id);
    ncclComm_t c = nullptr;
    nccl_check(ncclCommInitRank(&c, size, id, rank), "ncclCommInitRank");
    comm_ = c;
}

RcclTransport::~RcclTransport() {
    if (buf_) (void)hipFree(buf_);
    if (comm_) (void)ncclCommDestroy((ncclComm_t)comm_);
}

// tickets: every rank's count, then every rank's rows padded to the largest count (two
// all-gathers of device buffers on the transport's stream; tickets are small)
int RcclTransport::AllGather(const std::vector<int64_t>& mine, std::vector<int64_t>& all) {
    hipStream_t s = (hipStream_t)stream_;
    auto reserve = [&](size_t words) {
        if (words <= buf_cap_) return true;
        if (buf_) (void)hipFree(buf_);
        buf_cap_ = words + words / 2 + 64;
        return hipMalloc((void**)&buf_, buf_cap_ * 8) == hipSuccess;
    };
    if (!reserve((size_t)2 * size_)) return NFK_ERR_HIP;
    const int64_t n = (int64_t)mine.size();
    if (hipMemcpyAsync(buf_, &n, 8, hipMemcpyHostToDevice, s) != hipSuccess) return NFK_ERR_HIP;
    if (ncclAllGather(buf_, buf_ + size_, 1, ncclInt64, (ncclComm_t)comm_, s) != ncclSuccess) return NFK_ERR_HIP;
    std::vector<int64_t> counts(size_);
    if (hipMemcpyAsync(counts.data(), buf_ + size_, 8 * (size_t)size_, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return NFK_ERR_HIP;
    int64_t mx = 0;
    for (int64_t c : counts) mx = std::max(mx, c);
    all.clear();
    if (mx == 0) return NFK_OK;
    if (!reserve((size_t)mx * (1 + size_))) return NFK_ERR_HIP;
    if ((n && hipMemcpyAsync(buf_, mine.data(), (size_t)n * 8, hipMemcpyHostToDevice, s) != hipSuccess) ||
        ncclAllGather(buf_, buf_ + mx, (size_t)mx, ncclInt64, (ncclComm_t)comm_, s) != ncclSuccess)
        return NFK_ERR_HIP;
    std::vector<int64_t> padded((size_t)mx * size_);
    if (hipMemcpyAsync(padded.data(), buf_ + mx, padded.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return NFK_ERR_HIP;
    for (int r = 0; r < size_; r++) all.insert(all.end(), padded.begin() + (size_t)r * mx, padded.begin() + (size_t)r * mx + counts[r]);
    return NFK_OK;
}

int RcclTransport::AllToAllV(const uint64_t* send, const std::vector<size_t>& scount, uint64_t* recv,
                             const std::vector<size_t>& rcount, void* stream) {
    hipStream_t s = (hipStream_t)(stream ? stream : stream_);
    size_t so = 0, ro = 0;
    if (ncclGroupStart() != ncclSuccess) return NFK_ERR_HIP;
    for (int r = 0; r < size_; r++) {
        if (scount[r] && ncclSend(send + so, scount[r], ncclUint64, r, (ncclComm_t)comm_, s) != ncclSuccess)
            return NFK_ERR_HIP;
        if (rcount[r] && ncclRecv(recv + ro, rcount[r], ncclUint64, r, (ncclComm_t)comm_, s) != ncclSuccess)
            return NFK_ERR_HIP;
        so += scount[r];
        ro += rcount[r];
    }
    if (ncclGroupEnd() != ncclSuccess) return NFK_ERR_HIP;
    return NFK_OK;
}

}  // namespace nfgpu
