// shard_protocol.cpp — the C++ scene-shard exchange (include/NFGPUSceneShard.hpp) at world size 2,
// ranks as two threads with the host stand-in transport.  Over the recording C-ABI stub
// (tests/cpp/_stub, CPU) it checks the protocol; over libnfgpu.so (a GPU box) the same program moves
// real device rows between two worlds on the one GPU.
//
// Each rank owns one scene and six entities (7, 100 * rank + i); its even entities SwitchScene into
// the other rank's scene (group 5 + i, position (i, 2i, 3i)).  After one Migrate every rank holds
// its odd entities and the other's even ones, the rows intact, and the arrivals got the SwitchScene
// property writes GroupID = 0, SceneID, X, Y, Z, GroupID (KM:930-942).
//
// usage: shard_protocol [host|device]   (exit 0 = every check passed)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "NFGPUSceneShard.hpp"
#include "nfgpu.h"

using namespace nfgpu;

static int g_fail = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "rank check failed: " __VA_ARGS__); \
            fprintf(stderr, "\n");                     \
            g_fail = 1;                                \
        }                                              \
    } while (0)

// schema: SceneID, GroupID, HP (int); X, Y, Z (f64)
enum { P_SCENE, P_GROUP, P_HP, P_X, P_Y, P_Z, NP };

static void* make_world(int rank) {
    nfk_config cfg{};
    cfg.capacity = 64;
    cfg.n_int = 3;
    cfg.n_flt = 3;
    cfg.n_class = 2;
    cfg.n_kind = 0;
    cfg.n_rec = 0;
    void* w = nullptr;
    if (nfk_create(&cfg, &w) != NFK_OK) return nullptr;
    const uint8_t fl[NP] = {2, 2, 1, 1, 1, 1};
    nfk_set_prop_flags(w, 0, fl);
    nfk_set_prop_flags(w, 1, fl);
    std::vector<int64_t> gh(6, 7), gd(6);
    std::vector<int32_t> sc(6, 1 + rank), gr(6);
    std::vector<uint8_t> cl(6, 0), pl(6, 0);
    for (int i = 0; i < 6; i++) {
        gd[i] = 100 * rank + i;
        gr[i] = 1 + i % 2;
    }
    nfk_create_objects(w, 6, gh.data(), gd.data(), sc.data(), gr.data(), cl.data(), pl.data());
    std::vector<uint64_t> v(6);
    for (int i = 0; i < 6; i++) v[i] = (uint64_t)(1 + rank);
    nfk_load_prop(w, P_SCENE, v.data());
    for (int i = 0; i < 6; i++) v[i] = (uint64_t)gr[i];
    nfk_load_prop(w, P_GROUP, v.data());
    for (int i = 0; i < 6; i++) v[i] = (uint64_t)(1000 * rank + 10 * i);
    nfk_load_prop(w, P_HP, v.data());
    for (int p = P_X; p <= P_Z; p++) {
        for (int i = 0; i < 6; i++) {
            const double d = 0.5 * (p - P_X + 1) + rank;
            memcpy(&v[i], &d, 8);
        }
        nfk_load_prop(w, p, v.data());
    }
    nfk_commit(w);
    nfk_set_scene_props(w, P_SCENE, P_GROUP, P_X, P_Y, P_Z);
    return w;
}

int main(int argc, char** argv) {
    const bool device = argc > 1 && std::string(argv[1]) == "device";
    void* worlds[2] = {make_world(0), make_world(1)};
    if (!worlds[0] || !worlds[1]) {
        fprintf(stderr, "nfk_create failed: %s\n", nfk_last_error());
        return 2;
    }
    auto shared = HostTransport::MakeShared(2);
    RowMemory mem = device ? DeviceRowMemory() : HostRowMemory();
    std::vector<Ticket> sent[2], recv[2];
    int rc[2] = {0, 0};
    auto rank_main = [&](int r) {
        HostTransport t(shared, r, mem);
        SceneShard sh(worlds[r], &t, [](int scene) { return scene == 1 ? 0 : 1; }, P_SCENE, P_GROUP, P_X, P_Y, P_Z,
                      mem);
        for (int i = 0; i < 6; i += 2) sh.QueueSwitch(7, 100 * r + i, 0, 0, 2 - r, 5 + i, (float)i, 2.0f * i, 3.0f * i);
        rc[r] = sh.Migrate(&sent[r], &recv[r]);
        // a frame with no tickets anywhere: nothing moves
        if (!rc[r]) {
            std::vector<Ticket> s2, r2;
            rc[r] = sh.Migrate(&s2, &r2);
            CHECK(s2.empty() && r2.empty(), "empty frame moved entities");
        }
        CHECK(sh.migrated_out == 3 && sh.migrated_in == 3, "counts %lld %lld", (long long)sh.migrated_out,
              (long long)sh.migrated_in);
    };
    std::thread t0(rank_main, 0), t1(rank_main, 1);
    t0.join();
    t1.join();
    CHECK(rc[0] == 0 && rc[1] == 0, "Migrate failed: %d %d (%s)", rc[0], rc[1], nfk_last_error());
    if (g_fail) return 1;
    for (int r = 0; r < 2; r++) {
        const int o = 1 - r;
        CHECK(sent[r].size() == 3 && recv[r].size() == 3, "rank %d tickets %zu %zu", r, sent[r].size(), recv[r].size());
        for (int k = 0; k < 3; k++) {
            const Ticket& t = recv[r][k];
            CHECK(t.guid_data == 100 * o + 2 * k && t.src == o && t.dst == r && t.scene == 1 + r && t.group == 5 + 2 * k,
                  "rank %d ticket %d", r, k);
        }
        // frame state as the next Execute would start it: read-your-writes through nfk_get_props
        for (int i = 0; i < 6; i++) {
            const bool mine = (i % 2) == 1;  // odd entities stayed
            const int64_t gd_mine = 100 * r + i, gd_arr = 100 * o + i;
            int64_t h = 7, d = mine ? gd_mine : gd_arr;
            int32_t pids[NP] = {P_SCENE, P_GROUP, P_HP, P_X, P_Y, P_Z};
            uint64_t got[NP];
            std::vector<int64_t> hh(NP, h), dd(NP, d);
            const int e = nfk_get_props(worlds[r], NP, hh.data(), dd.data(), pids, got);
            CHECK(e == NFK_OK, "rank %d entity %lld missing", r, (long long)d);
            if (e) continue;
            const int src = mine ? r : o;
            CHECK(got[P_HP] == (uint64_t)(1000 * src + 10 * i), "rank %d entity %lld HP %llu", r, (long long)d,
                  (unsigned long long)got[P_HP]);
            if (mine) {
                CHECK(got[P_SCENE] == (uint64_t)(1 + r), "rank %d kept entity scene", r);
            } else {
                double x, y, z;
                memcpy(&x, &got[P_X], 8);
                memcpy(&y, &got[P_Y], 8);
                memcpy(&z, &got[P_Z], 8);
                CHECK(got[P_SCENE] == (uint64_t)(1 + r) && got[P_GROUP] == (uint64_t)(5 + i) && x == (double)(float)i &&
                          y == 2.0 * i && z == 3.0 * i,
                      "rank %d arrival %lld: scene %llu group %llu x %g", r, (long long)d, (unsigned long long)got[P_SCENE],
                      (unsigned long long)got[P_GROUP], x);
            }
            // the departed entities are gone from the source
            int32_t p0 = P_HP;
            uint64_t b;
            int64_t gone_d = mine ? gd_arr : gd_mine;
            if (!mine) CHECK(nfk_get_props(worlds[r], 1, &h, &gone_d, &p0, &b) == NFK_ERR_NOTFOUND,
                             "rank %d still holds %lld", r, (long long)gone_d);
        }
    }
    nfk_destroy(worlds[0]);
    nfk_destroy(worlds[1]);
    if (g_fail) return g_fail;

    // ---- the per-frame protocol (BeginFrame / EndFrame) with an exchange every 3rd frame: tickets
    // queued in window 2 are gathered by frame 3's EndFrame (on a worker thread) and their rows move
    // at frame 4's BeginFrame; a frame that is not an exchange frame, or follows an empty gather,
    // makes no transport call at all ----
    void* w2[2] = {make_world(0), make_world(1)};
    auto shared2 = HostTransport::MakeShared(2);
    int64_t calls[2][10] = {}, moved[2] = {0, 0};
    auto rank_frames = [&](int r) {
        HostTransport t(shared2, r, mem);
        SceneShard sh(w2[r], &t, [](int scene) { return scene == 1 ? 0 : 1; }, P_SCENE, P_GROUP, P_X, P_Y, P_Z, mem);
        sh.SetExchangeEvery(3);
        for (int f = 1; f <= 9; f++) {
            const int64_t c0 = sh.transport_calls;
            if (f == 2) sh.QueueSwitch(7, 100 * r + 1, 0, 0, 2 - r, 9, 1.0f, 2.0f, 3.0f);
            std::vector<Ticket> s, rv;
            CHECK(sh.BeginFrame(&s, &rv) == NFK_OK, "rank %d BeginFrame %d", r, f);
            if (f == 4) CHECK(s.size() == 1 && rv.size() == 1, "rank %d frame 4 moved %zu %zu", r, s.size(), rv.size());
            else CHECK(s.empty() && rv.empty(), "rank %d frame %d moved entities", r, f);
            CHECK(sh.EndFrame() == NFK_OK, "rank %d EndFrame %d", r, f);
            calls[r][f] = sh.transport_calls - c0;
        }
        moved[r] = sh.migrated_out + sh.migrated_in;
    };
    std::thread f0(rank_frames, 0), f1(rank_frames, 1);
    f0.join();
    f1.join();
    const int64_t want[10] = {0, 0, 0, 1, 2, 0, 1, 0, 0, 1};
    for (int r = 0; r < 2; r++) {
        for (int f = 1; f <= 9; f++)
            CHECK(calls[r][f] == want[f], "rank %d frame %d: %lld transport calls, want %lld", r, f, (long long)calls[r][f],
                  (long long)want[f]);
        CHECK(moved[r] == 2, "rank %d moved %lld", r, (long long)moved[r]);
        int64_t h = 7, d = 100 * (1 - r) + 1;
        int32_t p = P_GROUP;
        uint64_t b = 0;
        CHECK(nfk_get_props(w2[r], 1, &h, &d, &p, &b) == NFK_OK && b == 9, "rank %d arrival group %llu", r,
              (unsigned long long)b);
    }
    nfk_destroy(w2[0]);
    nfk_destroy(w2[1]);

    // ---- a departure that cannot leave (no such entity on rank 0): every rank learns every rank's
    // export status before the row exchange, so both fail and neither waits for the other ----
    void* w3[2] = {make_world(0), make_world(1)};
    auto shared3 = HostTransport::MakeShared(2);
    int rc3[2] = {0, 0};
    auto rank_fail = [&](int r) {
        HostTransport t(shared3, r, mem);
        SceneShard sh(w3[r], &t, [](int scene) { return scene == 1 ? 0 : 1; }, P_SCENE, P_GROUP, P_X, P_Y, P_Z, mem);
        sh.QueueSwitch(7, r == 0 ? 999 : 101, 0, 0, 2 - r, 3, 0.f, 0.f, 0.f);
        rc3[r] = sh.Migrate();
    };
    std::thread g0(rank_fail, 0), g1(rank_fail, 1);
    g0.join();
    g1.join();
    CHECK(rc3[0] != NFK_OK && rc3[1] != NFK_OK, "a failed export: statuses %d %d", rc3[0], rc3[1]);
    nfk_destroy(w3[0]);
    nfk_destroy(w3[1]);

    // ---- teardown while a peer never arrives: rank 1 never joins rank 0's ticket gather; the
    // shard's destructor waits NFGPU_SHARD_TEARDOWN_S, then aborts the transport and returns ----
    {
        setenv("NFGPU_SHARD_TEARDOWN_S", "0.5", 1);
        void* w4 = make_world(0);
        auto shared4 = HostTransport::MakeShared(2);
        const auto t0 = std::chrono::steady_clock::now();
        {
            HostTransport t(shared4, 0, mem);
            SceneShard sh(w4, &t, [](int scene) { return scene == 1 ? 0 : 1; }, P_SCENE, P_GROUP, P_X, P_Y, P_Z, mem);
            sh.QueueSwitch(7, 0, 0, 0, 2, 3, 0.f, 0.f, 0.f);
            CHECK(sh.EndFrame() == NFK_OK, "EndFrame");
        }  // (~SceneShard: the gather is still waiting for rank 1)
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CHECK(s < 10.0, "teardown with an absent peer took %.1f s", s);
        nfk_destroy(w4);
    }
    if (!g_fail) printf("shard_protocol %s: ok\n", device ? "device" : "host");
    return g_fail;
}
