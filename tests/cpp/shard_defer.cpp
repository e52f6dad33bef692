// shard_defer.cpp — a cross-shard SwitchScene of an entity whose membership changed in the same
// window (spawned by CreateObject after AfterInit, or switched within its shard) through the C++
// plugin: its row cannot be exported before the frame applies that change (the library refuses,
// nfgpu_host.hip nfk_export_objects), so the plugin defers the departure to the end of the next
// device frame instead of failing every rank's exchange and losing the entity.  Two ranks as
// threads (rank 0 owns scene 1, rank 1 scene 2) joined by the host transport, each an
// NFGPUKernelModule over the stub world (argv[1] = "host") or a real one on the GPU ("device").
//   window 0, rank 0: CreateObject(E) in scene 1 and SwitchScene(E -> scene 2) (deferred);
//                     SwitchScene(F -> scene 1 group 4) then SwitchScene(F -> scene 2) (deferred);
//                     SwitchScene(G -> scene 2) for a settled entity (leaves at once)
//   both ranks: MigrateNow (G moves; E and F may not be exported yet), then three Executes
//   then rank 1 holds E, F, G with their rows (HP), rank 0 none of them.
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "NFGPUKernelModule.hpp"
#include "NFGPUSceneShard.hpp"

using namespace nfgpu;

static int g_fail = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "check failed: " __VA_ARGS__); \
            fprintf(stderr, "\n");                     \
            g_fail = 1;                                \
        }                                              \
    } while (0)

int main(int argc, char** argv) {
    const bool device = argc > 1 && std::string(argv[1]) == "device";
    auto shared = HostTransport::MakeShared(2);
    RowMemory mem = device ? DeviceRowMemory() : HostRowMemory();
    const NFGUID E(9, 500), F(9, 1), G(9, 2);
    int present[2][3] = {{-1, -1, -1}, {-1, -1, -1}};
    int64_t hp[3] = {0, 0, 0};
    int rc[2] = {0, 0};
    auto rank_main = [&](int r) {
        try {
            int64_t now = 1000;
            HostTransport t(shared, r, mem);
            NFGPUKernelModule km(64);
            km.SetTimeSource([&now] { return now; });
            for (const char* p : {"SceneID", "GroupID", "HP"}) km.AddProperty(p, TDATA_INT);
            for (const char* p : {"X", "Y", "Z"}) km.AddProperty(p, TDATA_FLOAT);
            km.AddClass("NPC");
            km.SetPropertyFlags("NPC", "HP", true, true, false);
            km.Init();
            km.CreateScene(r + 1);
            for (int i = 0; i < 4; i++) {
                std::map<std::string, TData> init;
                TData v;
                v.type = TDATA_INT;
                v.i = 100 * (r + 1) + i;
                init["HP"] = v;
                km.CreateObject(NFGUID(9 + r, i + 1), r + 1, 0, "NPC", init);
            }
            km.AfterInit();
            SceneShard shard(km.World(), &t, [](int scene) { return scene == 1 ? 0 : 1; }, km.PropertyId("SceneID"),
                             km.PropertyId("GroupID"), km.PropertyId("X"), km.PropertyId("Y"), km.PropertyId("Z"), mem);
            km.AttachShard(&shard);
            km.Execute();  // (a settled first frame)
            now += 100;
            if (r == 0) {
                std::map<std::string, TData> init;
                TData v;
                v.type = TDATA_INT;
                v.i = 777;
                init["HP"] = v;
                CHECK(km.CreateObject(E, 1, 0, "NPC", init), "CreateObject(E)");
                CHECK(km.SwitchScene(E, 2, 3, 1.f, 2.f, 3.f), "SwitchScene(E)");
                CHECK(km.SwitchScene(F, 1, 4, 0.f, 0.f, 0.f), "SwitchScene(F) within the shard");
                CHECK(km.SwitchScene(F, 2, 5, 0.f, 0.f, 0.f), "SwitchScene(F)");
                CHECK(km.SwitchScene(G, 2, 6, 0.f, 0.f, 0.f), "SwitchScene(G)");
                // G's departure is queued (it stays this module's until its row is exported); E and F
                // stay this module's until the frame applied their change
                CHECK(km.Departing(G) && km.ObjectIndex(G) >= 0 && !km.Departing(E) && !km.Departing(F) &&
                          km.ObjectIndex(E) >= 0 && km.ObjectIndex(F) >= 0, "after the calls");
                CHECK(!km.SwitchScene(G, 1, 2, 0.f, 0.f, 0.f) && !km.DestroyObject(G), "G in transit");
            }
            km.MigrateNow();  // G moves now; E and F would be refused by the export
            if (r == 0) CHECK(km.ObjectIndex(G) < 0 && !km.Departing(G), "G left");
            for (int f = 0; f < 3; f++) {
                km.Execute();
                now += 100;
            }
            const NFGUID gs[3] = {E, F, G};
            for (int i = 0; i < 3; i++) {
                present[r][i] = km.ObjectIndex(gs[i]) >= 0;
                if (r == 1 && present[r][i]) hp[i] = km.GetPropertyInt(gs[i], "HP");
            }
            if (r == 1 && present[r][0]) {
                CHECK(km.GetPropertyInt(E, "SceneID") == 2 && km.GetPropertyInt(E, "GroupID") == 3, "E's scene %lld %lld",
                      (long long)km.GetPropertyInt(E, "SceneID"), (long long)km.GetPropertyInt(E, "GroupID"));
            }
            km.Shut();
        } catch (const std::exception& ex) {
            fprintf(stderr, "rank %d: %s\n", r, ex.what());
            rc[r] = 1;
        }
    };
    std::thread t0(rank_main, 0), t1(rank_main, 1);
    t0.join();
    t1.join();
    CHECK(rc[0] == 0 && rc[1] == 0, "a rank failed");
    for (int i = 0; i < 3; i++)
        CHECK(present[0][i] == 0 && present[1][i] == 1, "entity %d: rank 0 %d rank 1 %d", i, present[0][i], present[1][i]);
    CHECK(hp[0] == 777 && hp[1] == 100 && hp[2] == 101, "rows %lld %lld %lld", (long long)hp[0], (long long)hp[1],
          (long long)hp[2]);
    if (!g_fail) printf("shard_defer %s: ok\n", device ? "device" : "host");
    return g_fail;
}
