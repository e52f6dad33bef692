// functor_frame.cpp — what a heartbeat functor's own calls do, through the plugin API.
//
// In NFCScheduleModule::Execute (SM:49-119) a functor runs inside the walk: its SetProperty calls
// land at once (their property events fire before Execute returns) and its AddSchedule /
// RemoveSchedule calls are applied at the end of the same walk.  NFGPUKernelModule runs the
// functors after the device frame and applies their calls with a second device pass in the same
// Execute (nfk_execute_calls); with SetFunctorCallsSameFrame(false) they land one frame later.
//
// usage: functor_frame <same_frame 0|1>     prints one line per observation (see
// tests/test_gpu_parity.py::test_functor_calls_land_in_the_same_frame)
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "NFGPUKernelModule.hpp"

using namespace nfgpu;

static int64_t g_now = 1'700'000'000'000;

int main(int argc, char** argv) {
    if (argc != 2) return 2;
    const bool same = atoi(argv[1]) != 0;
    NFGPUKernelModule km(64);
    km.SetTimeSource([] { return g_now; });
    km.SetFunctorCallsSameFrame(same);
    km.AddProperty("HP", TDATA_INT);
    km.AddProperty("Level", TDATA_INT);
    km.AddClass("NPC");
    km.AddClass("Player");
    for (const char* c : {"NPC", "Player"}) {
        km.SetPropertyFlags(c, "HP", true, true, false);
        km.SetPropertyFlags(c, "Level", true, true, false);
    }
    km.AddHeartBeatProgram("Bonus", {});  // functor-only heartbeats: no device effect
    km.AddHeartBeatProgram("Regen", {});
    km.Init();
    km.CreateScene(1);
    std::vector<NFGUID> g;
    for (int i = 0; i < 4; i++) {
        g.push_back(NFGUID(1, 100 + i));
        std::map<std::string, TData> init;
        TData hp;
        hp.type = TDATA_INT;
        hp.i = 10 * i;
        init["HP"] = hp;
        if (!km.CreateObject(g[i], 1, 0, i < 2 ? "Player" : "NPC", init)) return 3;
    }
    km.AfterInit();

    int frame = 0;
    km.RegisterCommonPropertyEvent([&](const NFGUID& self, const std::string& name, const TData& a, const TData& b) {
        printf("event frame=%d obj=%lld %s %lld->%lld\n", frame, (long long)self.nData64, name.c_str(),
               (long long)a.GetInt(), (long long)b.GetInt());
        return 0;
    });
    // Regen: HP += 1 (read-your-writes), and at its 2nd fire add a "Bonus" schedule whose functor
    // raises Level; the last fire of Regen removes nothing (count runs out by itself)
    OBJECT_SCHEDULE_FUNCTOR bonus = [&](const NFGUID& self, const std::string& name, float, int n) {
        printf("fire frame=%d obj=%lld %s remain=%d\n", frame, (long long)self.nData64, name.c_str(), n);
        km.SetPropertyInt(self, "Level", km.GetPropertyInt(self, "Level") + 1);
        return 0;
    };
    OBJECT_SCHEDULE_FUNCTOR regen = [&](const NFGUID& self, const std::string& name, float, int n) {
        printf("fire frame=%d obj=%lld %s remain=%d\n", frame, (long long)self.nData64, name.c_str(), n);
        km.SetPropertyInt(self, "HP", km.GetPropertyInt(self, "HP") + 1);
        if (n == 2) km.AddSchedule(self, "Bonus", bonus, 0.05f, 2);
        return 0;
    };
    for (int i = 0; i < 2; i++) km.AddSchedule(g[i], "Regen", regen, 0.1f, 3);
    for (frame = 0; frame < 6; frame++) {
        g_now += 100;
        km.Execute();
        for (int i = 0; i < 2; i++)
            printf("state frame=%d obj=%lld HP=%lld Level=%lld Bonus=%d\n", frame, (long long)g[i].nData64,
                   (long long)km.GetPropertyInt(g[i], "HP"), (long long)km.GetPropertyInt(g[i], "Level"),
                   (int)km.ExistSchedule(g[i], "Bonus"));
    }
    km.Shut();
    return 0;
}
