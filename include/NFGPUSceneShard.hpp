// NFGPUSceneShard.hpp — scene shards across GPUs for a C++ game server, the C++
// counterpart of noahgameframe_amd/shard.py.
//
// One process per GPU owns a range of scenes and runs its own world; a scene group never spans two
// shards, so frames need no collective.  The only exchange on the path is a SwitchScene
// (NFCKernelModule::SwitchScene, KM:901-951) into a scene another shard owns: the entity's state
// row leaves the source world (nfk_export_objects), travels with one all-to-all per frame (RCCL
// over xGMI: ncclSend / ncclRecv on the world's stream, device to device), and enters the owner's
// world (nfk_import_objects), where the SwitchScene property writes follow (GroupID = 0, SceneID,
// X, Y, Z, GroupID; KM:930-942), so that frame's events come from the new scene group as on a
// single world.  Tickets (which entity goes where) are all-gathered first; a frame with no ticket
// anywhere moves nothing else.
//
// Transports: RcclTransport (librccl, one rank per GPU, the production path) and HostTransport
// (ranks as threads of one process exchanging through shared host memory: the protocol test's
// stand-in, tests/cpp/shard_protocol.cpp).
//
// Per frame (NFGPUKernelModule::Execute, or a server loop of its own):
//   BeginFrame()  before the frame's device pass: finishes the ticket all-gather started at the end
//                 of the previous frame; when its plan is not empty, the departures' rows leave the
//                 world (nfk_export_objects), every rank's export status is all-gathered (so all
//                 ranks go on to the row exchange or all stop: a failed export never leaves a peer
//                 waiting in a collective), the rows move and the arrivals enter with their
//                 SwitchScene property writes.  An empty plan makes no collective at all.
//   EndFrame()    after the frame: on an exchange frame (every `exchange_every`-th, the same on
//                 every rank) starts the all-gather of the tickets queued so far on a worker thread
//                 and the transport's side channel (RCCL: a communicator split off the rows' one, on
//                 its own stream), so it runs while the game logic prepares the next frame; on other
//                 frames it makes no transport call.
// A SwitchScene into another shard therefore takes effect at the start of the frame after the
// next exchange frame.  Migrate() is the synchronous form (gather now, rows now).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <future>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace nfgpu {

// one cross-shard SwitchScene; on the wire an int64[11] row (x, y, z as f64 bit patterns)
struct Ticket {
    int64_t guid_head = 0, guid_data = 0;
    int32_t cls = 0, is_player = 0, scene = 0, group = 0;
    double x = 0, y = 0, z = 0;
    int32_t src = -1, dst = -1;
};
constexpr int kTicketWords = 11;

// where rows live (device memory for a GPU world; host memory for a host stand-in world)
struct RowMemory {
    std::function<void*(size_t)> alloc;
    std::function<void(void*)> release;
    // copy between two row buffers of this memory (host stand-in transports use it)
    std::function<void(void*, const void*, size_t)> copy;
};
RowMemory DeviceRowMemory();  // hipMalloc / hipFree / hipMemcpy device to device
inline RowMemory HostRowMemory() {
    return RowMemory{[](size_t n) { return (void*)new uint8_t[n ? n : 1]; }, [](void* p) { delete[] (uint8_t*)p; },
                     [](void* d, const void* s, size_t n) {
                         for (size_t i = 0; i < n; i++) ((uint8_t*)d)[i] = ((const uint8_t*)s)[i];
                     }};
}

class ShardTransport {
public:
    virtual ~ShardTransport() = default;
    virtual int Rank() const = 0;
    virtual int Size() const = 0;
    // every rank's int64 words, concatenated in rank order (collective; the tickets' channel, which
    // may run on a worker thread while the rows' channel is idle)
    virtual int AllGather(const std::vector<int64_t>& mine, std::vector<int64_t>& all) = 0;
    // rows: send[r] / recv[r] words to / from rank r, buffers packed in rank order (collective);
    // stream: the world's stream (RCCL enqueues there; host transports wait for it first)
    virtual int AllToAllV(const uint64_t* send, const std::vector<size_t>& scount, uint64_t* recv,
                          const std::vector<size_t>& rcount, void* stream) = 0;
    // the rows must be complete in memory before AllToAllV (host transports)
    virtual bool NeedsHostSync() const = 0;
    // after an error, or when a peer never arrives: make a collective this rank is blocked in (or
    // enters later) return an error instead of waiting; the transport is unusable afterwards
    virtual void Abort() {}
};

// Ranks as threads of one process: every collective meets at a barrier in shared state.
class HostTransport : public ShardTransport {
public:
    struct Shared;
    static std::shared_ptr<Shared> MakeShared(int size);
    HostTransport(std::shared_ptr<Shared> s, int rank, RowMemory mem);
    int Rank() const override { return rank_; }
    int Size() const override;
    int AllGather(const std::vector<int64_t>& mine, std::vector<int64_t>& all) override;
    int AllToAllV(const uint64_t* send, const std::vector<size_t>& scount, uint64_t* recv,
                  const std::vector<size_t>& rcount, void* stream) override;
    bool NeedsHostSync() const override { return true; }
    void Abort() override;  // every rank's barrier returns an error from now on

private:
    std::shared_ptr<Shared> s_;
    int rank_;
    RowMemory mem_;
};

// RCCL (ncclComm per process, one GPU each): rows by grouped ncclSend / ncclRecv on the world's
// stream (the stream AllToAllV is given); tickets by ncclAllGather (count, then the rows padded to
// the largest count) on a communicator split off the rows' one and a stream of its own, so a ticket
// gather on a worker thread neither waits for nor blocks the world's stream.
class RcclTransport : public ShardTransport {
public:
    // unique_id: the 128-byte ncclUniqueId rank 0 made (NewUniqueId) and every rank received out
    // of band (the game server's own cluster channel)
    static std::vector<uint8_t> NewUniqueId();
    RcclTransport(const std::vector<uint8_t>& unique_id, int rank, int size, void* stream);
    ~RcclTransport() override;
    int Rank() const override { return rank_; }
    int Size() const override { return size_; }
    int AllGather(const std::vector<int64_t>& mine, std::vector<int64_t>& all) override;
    int AllToAllV(const uint64_t* send, const std::vector<size_t>& scount, uint64_t* recv,
                  const std::vector<size_t>& rcount, void* stream) override;
    bool NeedsHostSync() const override { return false; }
    void Abort() override;  // ncclCommAbort of both communicators

private:
    void* comm_ = nullptr;       // rows
    void* meta_comm_ = nullptr;  // tickets
    // set by Abort (possibly while the gather thread is inside a collective): the handles stay as they
    // are — the collective paths check this flag first, and the destructor, which runs after the
    // gather has been waited for, does not destroy communicators Abort has already released
    std::atomic<bool> aborted_{false};
    void* stream_ = nullptr;     // rows, when AllToAllV is given no stream
    void* meta_stream_ = nullptr;
    int device_ = 0;
    int rank_, size_;
    int64_t* buf_ = nullptr;  // device staging of the ticket all-gather
    size_t buf_cap_ = 0;
    // words of every rank's list gathered in the all-gather's first round, with its count: one
    // collective and one synchronisation when no rank has more (a second round gathers the rest).
    // It grows with the largest list seen (every rank sees the same lists: it is the same on all)
    size_t w_first_ = 16;
    int64_t* host_ = nullptr;  // pinned landing area of the gathers
    size_t host_cap_ = 0;
};

class SceneShard {
public:
    // owner(scene) -> rank; scene-property ids of the world (nfk_set_scene_props; -1: absent);
    // stream: the world's stream (nullptr: asked from the world, nfk_get_stream)
    SceneShard(void* world, ShardTransport* t, std::function<int(int)> owner, int pid_scene, int pid_group, int pid_x,
               int pid_y, int pid_z, RowMemory mem = DeviceRowMemory(), void* stream = nullptr);
    ~SceneShard();
    bool Owns(int scene) const { return owner_(scene) == t_->Rank(); }
    int Owner(int scene) const { return owner_(scene); }
    // a SwitchScene whose target this shard does not own: queued for the next exchange (the entity
    // leaves when that exchange's rows move)
    void QueueSwitch(int64_t guid_head, int64_t guid_data, int cls, int is_player, int scene, int group, float x,
                     float y, float z);
    // tickets are all-gathered every `every`-th EndFrame (the same on every rank; default 1)
    void SetExchangeEvery(int every) { every_ = every < 1 ? 1 : every; }
    // collective, before every frame on every rank (see the header): the rows of the plan gathered
    // one frame ago.  sent / received: this rank's tickets of that plan.
    int BeginFrame(std::vector<Ticket>* sent = nullptr, std::vector<Ticket>* received = nullptr);
    // collective, after every frame on every rank: starts the next ticket gather on an exchange frame
    int EndFrame();
    // synchronous exchange of the tickets queued so far (collective): gather, then rows
    int Migrate(std::vector<Ticket>* sent = nullptr, std::vector<Ticket>* received = nullptr);
    // NFIRankRedisModule::GetRange(type, 0, k - 1) over every shard's entities
    // (NFCRankRedisModule.cpp:109-118: a ZREVRANGE WITH SCORES of the whole key) with a property as the
    // score: each rank's exact top k (nfk_rank_top on its world), all-gathered over the transport and
    // merged in ZREVRANGE order — score descending, equal scores by member NFGUID::ToString()
    // ("head-data", NFGUID.h:93) descending.  Collective (every rank calls it with the same pid and k,
    // in the same order relative to its Execute; a ticket gather EndFrame started is waited for first).
    struct RankRow {
        int64_t guid_head, guid_data;
        double score;
    };
    int RankTop(int pid, int k, std::vector<RankRow>* out);
    int64_t migrated_out = 0, migrated_in = 0;
    int64_t transport_calls = 0;  // collective calls this shard made (AllGather, AllToAllV)
    int64_t frames = 0;           // EndFrame calls

private:
    std::vector<int64_t> TakeTickets();
    int Rows(const std::vector<int64_t>& plan, std::vector<Ticket>* sent, std::vector<Ticket>* received);
    void* world_;
    ShardTransport* t_;
    std::function<int(int)> owner_;
    int pid_scene_, pid_group_, pid_x_, pid_y_, pid_z_;
    RowMemory mem_;
    void* stream_;
    std::vector<Ticket> out_;
    uint64_t* sbuf_ = nullptr;
    uint64_t* rbuf_ = nullptr;
    size_t scap_ = 0, rcap_ = 0;
    int every_ = 1;
    std::future<int> pending_;  // the ticket gather started by the last exchange EndFrame
    bool failed_ = false;       // a transport call of this shard returned an error
    std::vector<int64_t> pending_plan_;
    // the gathers run on one persistent worker thread (started by the first exchange): a thread per
    // gather (std::async) cost its creation, and the HIP device's set-up on it, on every exchange frame
    void GatherLoop();
    std::thread worker_;
    std::mutex wmu_;
    std::condition_variable wcv_;
    bool wstop_ = false, wjob_ = false;
    std::vector<int64_t> wmine_;
    std::promise<int> wprom_;
};

}  // namespace nfgpu
