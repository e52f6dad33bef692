// shard_rank.cpp — the cross-shard leaderboard of the C++ scene shards (SceneShard::RankTop,
// NFGPUKernelModule::GetRange with a shard attached): NFIRankRedisModule::GetRange(type, 0, k - 1)
// over every shard's entities (NFCRankRedisModule.cpp:109-118, a ZREVRANGE WITH SCORES of the whole
// key).  R ranks as threads with the host stand-in transport, each with its own world holding the
// entities of the scenes it owns; one more world holds all of them.  Every rank's RankTop must equal
// that single world's nfk_rank_top, for an int and an f64 property with ties and k below, at and above
// the entity count.  Over the recording C-ABI stub (tests/cpp/_stub, CPU) or libnfgpu.so (a GPU box).
//
// usage: shard_rank <ranks>   (exit 0 = every check passed)
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "NFGPUSceneShard.hpp"
#include "nfgpu.h"

using namespace nfgpu;

static int g_fail = 0;
enum { P_SCENE, P_GROUP, P_GOLD, P_X, NP };  // SceneID, GroupID, Gold (int); X (f64)
constexpr int kPerScene = 150, kScenes = 8;

struct Ent {
    int64_t h, d;
    int32_t scene;
    int64_t gold;
    double x;
};

static void* make_world(const std::vector<Ent>& es) {
    nfk_config cfg{};
    cfg.capacity = (int32_t)es.size() + 64;
    cfg.n_int = 3;
    cfg.n_flt = 1;
    cfg.n_class = 1;
    void* w = nullptr;
    if (nfk_create(&cfg, &w) != NFK_OK) return nullptr;
    const uint8_t fl[NP] = {2, 2, 1, 1};
    nfk_set_prop_flags(w, 0, fl);
    const size_t n = es.size();
    std::vector<int64_t> gh(n), gd(n);
    std::vector<int32_t> sc(n), gr(n, 1);
    std::vector<uint8_t> cl(n, 0), pl(n, 0);
    std::vector<uint64_t> vs(n), vg(n), vo(n), vx(n);
    for (size_t i = 0; i < n; i++) {
        gh[i] = es[i].h;
        gd[i] = es[i].d;
        sc[i] = es[i].scene;
        vs[i] = (uint64_t)es[i].scene;
        vg[i] = 1;
        vo[i] = (uint64_t)es[i].gold;
        memcpy(&vx[i], &es[i].x, 8);
    }
    nfk_create_objects(w, (int32_t)n, gh.data(), gd.data(), sc.data(), gr.data(), cl.data(), pl.data());
    nfk_load_prop(w, P_SCENE, vs.data());
    nfk_load_prop(w, P_GROUP, vg.data());
    nfk_load_prop(w, P_GOLD, vo.data());
    nfk_load_prop(w, P_X, vx.data());
    if (nfk_commit(w) != NFK_OK) return nullptr;
    return w;
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 2;
    std::mt19937_64 rng(1234 + R);
    std::vector<Ent> all;
    for (int s = 1; s <= kScenes; s++)
        for (int i = 0; i < kPerScene; i++) {
            Ent e;
            e.h = (rng() & 1) ? 7 : 19;                       // members "7-..." and "19-...": string order
            e.d = (int64_t)(rng() % 100000) * 10 + s;         // is not numeric order
            e.scene = s;
            e.gold = (int64_t)(rng() % 40) * 25 - 300;        // many ties, negatives
            e.x = (double)(int64_t)(rng() % 64) * 0.5 - 8.0;  // ties in f64
            all.push_back(e);
        }
    auto owner = [R](int scene) { return (scene - 1) * R / kScenes; };
    void* whole = make_world(all);
    if (!whole) {
        fprintf(stderr, "world: %s\n", nfk_last_error());
        return 2;
    }
    struct Q {
        int pid, k;
    };
    const Q qs[] = {{P_GOLD, 10}, {P_GOLD, 333}, {P_X, 1}, {P_X, 57}, {P_GOLD, (int)all.size() + 5}};
    std::vector<std::vector<SceneShard::RankRow>> expect;
    for (const Q& q : qs) {
        std::vector<int64_t> gh((size_t)q.k), gd((size_t)q.k);
        std::vector<double> sc((size_t)q.k);
        int32_t n = 0;
        if (nfk_rank_top(whole, q.pid, q.k, &n, gh.data(), gd.data(), sc.data()) != NFK_OK) return 3;
        std::vector<SceneShard::RankRow> e;
        for (int32_t i = 0; i < n; i++) e.push_back({gh[(size_t)i], gd[(size_t)i], sc[(size_t)i]});
        expect.push_back(e);
    }
    auto shared = HostTransport::MakeShared(R);
    std::vector<int> rc(R, 0);
    auto rank_main = [&](int r) {
        std::vector<Ent> mine;
        for (const Ent& e : all)
            if (owner(e.scene) == r) mine.push_back(e);
        void* w = make_world(mine);
        if (!w) {
            rc[r] = 2;
            return;
        }
        HostTransport t(shared, r, HostRowMemory());
        SceneShard shard(w, &t, owner, P_SCENE, P_GROUP, P_X, -1, -1, HostRowMemory());
        for (size_t qi = 0; qi < sizeof(qs) / sizeof(qs[0]); qi++) {
            std::vector<SceneShard::RankRow> got;
            if (shard.RankTop(qs[qi].pid, qs[qi].k, &got) != NFK_OK) {
                rc[r] = 4;
                continue;
            }
            bool same = got.size() == expect[qi].size();
            for (size_t i = 0; same && i < got.size(); i++)
                same = got[i].guid_head == expect[qi][i].guid_head && got[i].guid_data == expect[qi][i].guid_data &&
                       got[i].score == expect[qi][i].score;
            if (!same) {
                fprintf(stderr, "rank %d query %zu: %zu rows, expected %zu\n", r, qi, got.size(), expect[qi].size());
                rc[r] = 5;
            }
        }
        nfk_destroy(w);
    };
    std::vector<std::thread> th;
    for (int r = 0; r < R; r++) th.emplace_back(rank_main, r);
    for (auto& x : th) x.join();
    nfk_destroy(whole);
    for (int r = 0; r < R; r++)
        if (rc[r]) g_fail = rc[r];
    if (!g_fail) printf("shard_rank %d ranks: ok (%zu entities, %zu queries)\n", R, all.size(), expect.size());
    return g_fail;
}
