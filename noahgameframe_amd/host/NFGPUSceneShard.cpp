// NFGPUSceneShard.cpp — the cross-shard SwitchScene exchange (include/NFGPUSceneShard.hpp) and the
// host stand-in transport.  RCCL lives in NFGPUShardRccl.cpp.
#include "NFGPUSceneShard.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>

#include "nfgpu.h"

namespace nfgpu {

// ---------------- HostTransport ----------------
struct HostTransport::Shared {
    int size;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t generation = 0;
    bool aborted = false;  // HostTransport::Abort: every barrier returns false
    std::vector<const std::vector<int64_t>*> gather_in;
    std::vector<const uint64_t*> send;
    std::vector<const std::vector<size_t>*> scount;
    // a barrier every rank passes; fn runs on the last arrival, before anyone leaves; false once
    // aborted (a rank that died or left never arrives)
    bool barrier(const std::function<void()>& fn = nullptr) {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return false;
        const int64_t g = generation;
        if (++arrived == size) {
            if (fn) fn();
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != g || aborted; });
        }
        return generation != g;
    }
};

std::shared_ptr<HostTransport::Shared> HostTransport::MakeShared(int size) {
    auto s = std::make_shared<Shared>();
    s->size = size;
    s->gather_in.assign(size, nullptr);
    s->send.assign(size, nullptr);
    s->scount.assign(size, nullptr);
    return s;
}

HostTransport::HostTransport(std::shared_ptr<Shared> s, int rank, RowMemory mem)
    : s_(std::move(s)), rank_(rank), mem_(std::move(mem)) {}

int HostTransport::Size() const { return s_->size; }

int HostTransport::AllGather(const std::vector<int64_t>& mine, std::vector<int64_t>& all) {
    {
        std::lock_guard<std::mutex> lk(s_->mu);
        s_->gather_in[rank_] = &mine;
    }
    if (!s_->barrier()) return NFK_ERR_STATE;  // every rank's input is published
    all.clear();
    for (int r = 0; r < s_->size; r++) all.insert(all.end(), s_->gather_in[r]->begin(), s_->gather_in[r]->end());
    if (!s_->barrier()) return NFK_ERR_STATE;  // every rank has read (the inputs may go)
    return NFK_OK;
}

void HostTransport::Abort() {
    std::lock_guard<std::mutex> lk(s_->mu);
    s_->aborted = true;
    s_->cv.notify_all();
}

int HostTransport::AllToAllV(const uint64_t* send, const std::vector<size_t>& scount, uint64_t* recv,
                             const std::vector<size_t>& rcount, void*) {
    {
        std::lock_guard<std::mutex> lk(s_->mu);
        s_->send[rank_] = send;
        s_->scount[rank_] = &scount;
    }
    if (!s_->barrier()) return NFK_ERR_STATE;
    // pull my part of every source's buffer: source r packs its rows in destination order
    int rc = NFK_OK;
    size_t at = 0;
    for (int r = 0; r < s_->size && rc == NFK_OK; r++) {
        const std::vector<size_t>& sc = *s_->scount[r];
        size_t off = 0;
        for (int q = 0; q < rank_; q++) off += sc[q];
        if (sc[rank_] != rcount[r]) {
            rc = NFK_ERR_STATE;  // (still through the second barrier: the peers are waiting at it)
            break;
        }
        if (rcount[r]) mem_.copy(recv + at, s_->send[r] + off, rcount[r] * 8);
        at += rcount[r];
    }
    if (!s_->barrier()) return NFK_ERR_STATE;
    return rc;
}

// ---------------- SceneShard ----------------
SceneShard::SceneShard(void* world, ShardTransport* t, std::function<int(int)> owner, int pid_scene, int pid_group,
                       int pid_x, int pid_y, int pid_z, RowMemory mem, void* stream)
    : world_(world), t_(t), owner_(std::move(owner)), pid_scene_(pid_scene), pid_group_(pid_group), pid_x_(pid_x),
      pid_y_(pid_y), pid_z_(pid_z), mem_(std::move(mem)), stream_(stream) {
    // the rows are packed and unpacked on the world's stream: an RCCL transport sends and receives
    // on that same stream (stream order, no host synchronisation)
    if (!stream_ && world_) (void)nfk_get_stream(world_, &stream_);
}

SceneShard::~SceneShard() {
    // A gather still in flight: the peers need this rank in it, so it is waited for — but not
    // forever.  After an error of this shard, or when it has not finished within
    // NFGPU_SHARD_TEARDOWN_S seconds (default 30: a peer that died never arrives), the transport
    // is aborted so that the collective returns and teardown completes.
    if (pending_.valid()) {
        const char* e = getenv("NFGPU_SHARD_TEARDOWN_S");
        const double secs = failed_ ? 0.0 : (e ? atof(e) : 30.0);
        if (pending_.wait_for(std::chrono::duration<double>(secs)) != std::future_status::ready) t_->Abort();
        (void)pending_.get();
    }
    if (worker_.joinable()) {  // (idle now: its last gather has been taken)
        {
            std::lock_guard<std::mutex> lk(wmu_);
            wstop_ = true;
        }
        wcv_.notify_one();
        worker_.join();
    }
    if (sbuf_) mem_.release(sbuf_);
    if (rbuf_) mem_.release(rbuf_);
}

void SceneShard::QueueSwitch(int64_t gh, int64_t gd, int cls, int is_player, int scene, int group, float x, float y,
                             float z) {
    Ticket k;
    k.guid_head = gh;
    k.guid_data = gd;
    k.cls = cls;
    k.is_player = is_player;
    k.scene = scene;
    k.group = group;
    k.x = (double)x;  // SwitchScene takes floats (KM:901); the properties are doubles
    k.y = (double)y;
    k.z = (double)z;
    k.src = t_->Rank();
    k.dst = owner_(scene);
    out_.push_back(k);
}

static uint64_t f64_bits(double v) {
    uint64_t b;
    memcpy(&b, &v, 8);
    return b;
}
static double bits_f64(int64_t b) {
    double v;
    memcpy(&v, &b, 8);
    return v;
}

// this rank's queued tickets as words (TICKET layout), taken off the queue
std::vector<int64_t> SceneShard::TakeTickets() {
    std::vector<int64_t> mine;
    mine.reserve(out_.size() * kTicketWords);
    for (const Ticket& k : out_) {
        const int64_t w[kTicketWords] = {k.guid_head, k.guid_data, k.cls, k.is_player, k.scene, k.group,
                                         (int64_t)f64_bits(k.x), (int64_t)f64_bits(k.y), (int64_t)f64_bits(k.z),
                                         k.src, k.dst};
        mine.insert(mine.end(), w, w + kTicketWords);
    }
    out_.clear();
    return mine;
}

int SceneShard::EndFrame() {
    frames++;
    if (pending_.valid()) return NFK_ERR_STATE;  // the last gather was never taken by BeginFrame
    if (frames % every_) return NFK_OK;          // not an exchange frame: no transport call
    std::vector<int64_t> mine = TakeTickets();
    transport_calls++;
    pending_plan_.clear();
    // on the worker thread: the game logic of the next window runs meanwhile
    std::promise<int> pr;
    pending_ = pr.get_future();
    {
        std::lock_guard<std::mutex> lk(wmu_);
        if (!worker_.joinable()) worker_ = std::thread(&SceneShard::GatherLoop, this);
        wmine_ = std::move(mine);
        wprom_ = std::move(pr);
        wjob_ = true;
    }
    wcv_.notify_one();
    return NFK_OK;
}

void SceneShard::GatherLoop() {
    std::unique_lock<std::mutex> lk(wmu_);
    for (;;) {
        wcv_.wait(lk, [this] { return wstop_ || wjob_; });
        if (!wjob_) return;  // (stopped, nothing queued)
        wjob_ = false;
        std::vector<int64_t> mine = std::move(wmine_);
        std::promise<int> pr = std::move(wprom_);
        lk.unlock();
        int r;
        try {
            r = t_->AllGather(mine, pending_plan_);
        } catch (...) {
            r = NFK_ERR_HIP;
        }
        pr.set_value(r);
        lk.lock();
    }
}

int SceneShard::BeginFrame(std::vector<Ticket>* sent, std::vector<Ticket>* received) {
    if (sent) sent->clear();
    if (received) received->clear();
    if (!pending_.valid()) return NFK_OK;  // no gather since the last one: nothing to move
    static const bool trace = getenv("NFGPU_TRACE_SHARD") != nullptr;
    const auto tw = std::chrono::steady_clock::now();
    const int r = pending_.get();
    if (trace)
        fprintf(stderr, "shard begin: ticket gather waited %.3f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tw).count());
    if (r) {
        failed_ = true;
        return r;
    }
    std::vector<int64_t> plan;
    plan.swap(pending_plan_);
    const int rr = Rows(plan, sent, received);
    if (rr) failed_ = true;
    return rr;
}

int SceneShard::Migrate(std::vector<Ticket>* sent, std::vector<Ticket>* received) {
    // (a gather EndFrame started is finished first: every rank makes its collectives in one order)
    std::vector<Ticket> s0, r0;
    int r = BeginFrame(&s0, &r0);
    if (r) return r;
    std::vector<int64_t> plan;
    transport_calls++;
    r = t_->AllGather(TakeTickets(), plan);
    if (r) {
        failed_ = true;
        return r;
    }
    r = Rows(plan, sent, received);
    if (r) failed_ = true;
    if (sent) sent->insert(sent->begin(), s0.begin(), s0.end());
    if (received) received->insert(received->begin(), r0.begin(), r0.end());
    return r;
}

// ZREVRANGE order of two leaderboard rows: score descending, then member NFGUID::ToString() descending
static bool zrev_before(const SceneShard::RankRow& a, const SceneShard::RankRow& b) {
    if (a.score != b.score) return a.score > b.score;
    const std::string ma = std::to_string(a.guid_head) + "-" + std::to_string(a.guid_data);
    const std::string mb = std::to_string(b.guid_head) + "-" + std::to_string(b.guid_data);
    return ma > mb;
}

int SceneShard::RankTop(int pid, int k, std::vector<RankRow>* out) {
    out->clear();
    if (k < 0) k = 0;
    std::vector<int64_t> gh((size_t)k + 1), gd((size_t)k + 1);
    std::vector<double> sc((size_t)k + 1);
    int32_t n = 0;
    const int status = k ? nfk_rank_top(world_, pid, k, &n, gh.data(), gd.data(), sc.data()) : NFK_OK;
    // (this rank's collectives in one order on every rank: the ticket gather in flight finishes first;
    // BeginFrame still takes its plan)
    if (pending_.valid()) pending_.wait();
    // [count (-1: this rank failed), then head, data, score bits per row]
    std::vector<int64_t> mine(1, status ? -1 : (int64_t)n), all;
    for (int32_t i = 0; !status && i < n; i++) {
        mine.push_back(gh[(size_t)i]);
        mine.push_back(gd[(size_t)i]);
        mine.push_back((int64_t)f64_bits(sc[(size_t)i]));
    }
    transport_calls++;
    const int r = t_->AllGather(mine, all);
    if (r) return r;
    int bad = 0;
    for (size_t at = 0; at < all.size();) {
        const int64_t c = all[at++];
        if (c < 0) {
            bad = 1;
            continue;
        }
        for (int64_t i = 0; i < c && at + 3 <= all.size(); i++, at += 3)
            out->push_back({all[at], all[at + 1], bits_f64(all[at + 2])});
    }
    if (status || bad) {
        out->clear();
        return status ? status : NFK_ERR_STATE;  // (a peer's nfk_rank_top failed)
    }
    std::stable_sort(out->begin(), out->end(), zrev_before);
    if ((int)out->size() > k) out->resize((size_t)k);
    return NFK_OK;
}

// the rows of a global plan (every rank's tickets in (source rank, call) order), rank to rank
int SceneShard::Rows(const std::vector<int64_t>& plan, std::vector<Ticket>* sent, std::vector<Ticket>* received) {
    const int ws = t_->Size(), me = t_->Rank();
    const size_t n = plan.size() / kTicketWords;
    if (n == 0) return NFK_OK;  // the same on every rank: no row exchange
    auto tk = [&](size_t i) {
        const int64_t* w = &plan[i * kTicketWords];
        Ticket k;
        k.guid_head = w[0];
        k.guid_data = w[1];
        k.cls = (int32_t)w[2];
        k.is_player = (int32_t)w[3];
        k.scene = (int32_t)w[4];
        k.group = (int32_t)w[5];
        k.x = bits_f64(w[6]);
        k.y = bits_f64(w[7]);
        k.z = bits_f64(w[8]);
        k.src = (int32_t)w[9];
        k.dst = (int32_t)w[10];
        return k;
    };
    // (NFGPU_TRACE_SHARD=1: this exchange's host phases on stderr)
    static const bool trace = getenv("NFGPU_TRACE_SHARD") != nullptr;
    using clk = std::chrono::steady_clock;
    clk::time_point tp[6];
    tp[0] = clk::now();
    std::vector<Ticket> snd, rcv;
    for (size_t i = 0; i < n; i++) {
        const Ticket k = tk(i);
        if (k.src == me) snd.push_back(k);
        if (k.dst == me) rcv.push_back(k);
    }
    // rows in destination order (call order within one), received in source order
    std::stable_sort(snd.begin(), snd.end(), [](const Ticket& a, const Ticket& b) { return a.dst < b.dst; });
    std::stable_sort(rcv.begin(), rcv.end(), [](const Ticket& a, const Ticket& b) { return a.src < b.src; });
    // 1. the local half: buffers and the export (the entities leave this world; rows packed on the
    // world's stream).  A failure here does not return yet: every rank first learns every rank's status
    int32_t rw = 0;
    int status = nfk_row_words(world_, &rw);
    std::vector<size_t> scount(ws, 0), rcount(ws, 0);
    if (!status) {
        for (const Ticket& k : snd) scount[k.dst] += (size_t)rw;
        for (const Ticket& k : rcv) rcount[k.src] += (size_t)rw;
        auto reserve = [&](uint64_t*& buf, size_t& cap, size_t words) {
            if (words <= cap) return;
            if (buf) mem_.release(buf);
            buf = nullptr;
            cap = 0;
            buf = (uint64_t*)mem_.alloc((words + words / 2 + 64) * 8);
            cap = words + words / 2 + 64;
        };
        try {
            reserve(sbuf_, scap_, snd.size() * (size_t)rw);
            reserve(rbuf_, rcap_, rcv.size() * (size_t)rw);
        } catch (const std::exception&) {
            status = NFK_ERR_HIP;
        }
    }
    if (!status && !snd.empty()) {
        std::vector<int64_t> gh(snd.size()), gd(snd.size());
        for (size_t i = 0; i < snd.size(); i++) {
            gh[i] = snd[i].guid_head;
            gd[i] = snd[i].guid_data;
        }
        status = nfk_export_objects(world_, (int32_t)snd.size(), gh.data(), gd.data(), sbuf_);
    }
    if (!status && t_->NeedsHostSync()) status = nfk_sync(world_);
    tp[1] = clk::now();
    // 2. every rank's status (collective): all ranks go on to the row exchange, or none does
    {
        std::vector<int64_t> mine(1, (int64_t)status), all;
        transport_calls++;
        const int r = t_->AllGather(mine, all);
        if (r) return r;
        for (int64_t v : all)
            if (v) return status ? status : NFK_ERR_STATE;  // (a peer failed: its rows never come)
    }
    tp[2] = clk::now();
    // 3. the rows, rank to rank (on the world's stream for RCCL)
    transport_calls++;
    int r = t_->AllToAllV(sbuf_, scount, rbuf_, rcount, stream_);
    if (r) return r;
    tp[3] = tp[4] = clk::now();
    // 4. import, then the SwitchScene property writes (KM:930-942): GroupID = 0, SceneID, X, Y, Z,
    // GroupID, per entity in this order (the scene always changes here)
    if (!rcv.empty()) {
        const size_t m = rcv.size();
        std::vector<int64_t> gh(m), gd(m);
        std::vector<int32_t> sc(m), gr(m);
        std::vector<uint8_t> cl(m), pl(m);
        for (size_t i = 0; i < m; i++) {
            gh[i] = rcv[i].guid_head;
            gd[i] = rcv[i].guid_data;
            sc[i] = rcv[i].scene;
            gr[i] = rcv[i].group;
            cl[i] = (uint8_t)rcv[i].cls;
            pl[i] = (uint8_t)rcv[i].is_player;
        }
        r = nfk_import_objects(world_, (int32_t)m, gh.data(), gd.data(), sc.data(), gr.data(), cl.data(), pl.data(),
                               rbuf_);
        if (r) return r;
        tp[4] = clk::now();
        std::vector<int64_t> wh, wd;
        std::vector<int32_t> wp;
        std::vector<uint64_t> wb;
        for (size_t i = 0; i < m; i++) {
            const std::pair<int, uint64_t> cols[6] = {
                {pid_group_, 0},
                {pid_scene_, (uint64_t)(int64_t)rcv[i].scene},
                {pid_x_, f64_bits(rcv[i].x)},
                {pid_y_, f64_bits(rcv[i].y)},
                {pid_z_, f64_bits(rcv[i].z)},
                {pid_group_, (uint64_t)(int64_t)rcv[i].group}};
            for (const auto& c : cols) {
                if (c.first < 0) continue;
                wh.push_back(gh[i]);
                wd.push_back(gd[i]);
                wp.push_back(c.first);
                wb.push_back(c.second);
            }
        }
        if (!wp.empty()) {
            r = nfk_set_props(world_, (int32_t)wp.size(), wh.data(), wd.data(), wp.data(), wb.data());
            if (r) return r;
        }
    }
    if (trace) {
        tp[5] = clk::now();
        auto ms = [&](int a, int b) { return std::chrono::duration<double, std::milli>(tp[b] - tp[a]).count(); };
        fprintf(stderr, "shard rows: %zu out %zu in: export %.3f ms, status gather %.3f ms, rows %.3f ms, import %.3f ms, "
                "writes %.3f ms\n", snd.size(), rcv.size(), ms(0, 1), ms(1, 2), ms(2, 3), ms(3, 4), ms(4, 5));
    }
    migrated_out += (int64_t)snd.size();
    migrated_in += (int64_t)rcv.size();
    if (sent) *sent = std::move(snd);
    if (received) *received = std::move(rcv);
    return NFK_OK;
}

}  // namespace nfgpu
