// tutorial3_session.cpp — the reference's Tutorial3 (Tutorial/Tutorial3/HelloWorld3Module.cpp and
// Tutorial3Plugin.cpp, compiled UNCHANGED where they lie) loaded by a NoahGameFrame server, once with the
// reference's own NFKernelPlugin (NFComm/NFKernelPlugin/NFKernelPlugin.cpp: NFCKernelModule,
// NFCSceneAOIModule, NFCEventModule, NFCScheduleModule; -DT3_REF) and once with the reference-side GPU
// plugin (integration/NFGPUKernelPlugin.cpp) in its place, with NFConfigPlugin (NFCClassModule,
// NFCElementModule) beside them.  The plugins are loaded and driven as NFCPluginManager does
// (NFPluginLoader/NFCPluginManager.cpp:60-93, 313-327, 472-481: plugins in name order, each plugin's
// modules in its map's order; FindModule strips the length prefix of typeid names, :440-465) on a
// virtual NFGetTime clock.
//
// Tutorial3's AfterInit creates scene 1, its class callback on Player, the object NFGUID(0, 10) with the
// dynamic properties Hello / World and their callbacks, and calls DoEvent.  Scaled to `objects` Player
// objects (NFGUID(0, 1000 + i), created a share per frame over the first 5 s so the 5 s heartbeats
// spread), each of which the tutorial's class callback gives OnEvent and the OnHeartBeat schedule
// (5 s x 10), and per frame DoEvent(1) on 1 % of them (the tutorial's OnEvent then sets Hello).  Everything
// the tutorial prints goes to stdout with a line per frame: the two servers' stdout must be equal
// (tests/test_tutorial3.py).  On the GPU plugin the heartbeat name OnHeartBeat is registered with an empty
// device program (what a logic module's Init does for a functor-only heartbeat): its
// timers are scanned on the device, its functor runs on the host in the walk's order.
//
// TEST INFRASTRUCTURE ONLY.  usage: tutorial3_session <objects> <frames> <tick_ms>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "NFComm/NFPluginModule/NFIPlugin.h"
#ifdef T3_REF
#include "NFComm/NFCore/NFCDataList.h"
#include "NFComm/NFKernelPlugin/NFKernelPlugin.h"
#include "NFComm/NFPluginModule/NFIEventModule.h"
#include "NFComm/NFPluginModule/NFIKernelModule.h"
#else
#include "../../integration/NFGPUKernelPlugin.cpp"
#endif
#include "NFComm/NFConfigPlugin/NFConfigPlugin.h"
#include "NFComm/NFMessageDefine/NFProtocolDefine.hpp"
#include "Tutorial/Tutorial3/Tutorial3Plugin.h"
#include "../../oracle/ref_server.hpp"

// NFGetTime() (NFPlatform.h:367) reads CLOCK_REALTIME: the session's virtual clock
extern "C" int clock_gettime(clockid_t clk, struct timespec* ts) {
    if (clk == CLOCK_REALTIME) {
        ts->tv_sec = g_now / 1000;
        ts->tv_nsec = (g_now % 1000) * 1000000;
        return 0;
    }
    return (int)syscall(SYS_clock_gettime, clk, ts);
}

// NFCPluginManager's plugin and module registry (NFCPluginManager.cpp:440-465: a typeid name's length
// prefix stripped; plugins kept by name)
class T3PluginManager : public TestPluginManager {
public:
    std::map<std::string, NFIPlugin*> plugins;
    using NFIPluginManager::FindModule;
    void Registered(NFIPlugin* p) override { plugins[p->GetPluginName()] = p; }
    NFIModule* FindModule(const std::string& n) override {
        std::string s = n;
        for (size_t i = 0; i < s.size(); i++) {
            const int len = atoi(s.substr(0, i + 1).c_str());
            if (s.size() == i + 1 + (size_t)len) {
                s = s.substr(i + 1);
                break;
            }
        }
        return TestPluginManager::FindModule(s);
    }
};

int main(int argc, char** argv) {
    if (argc != 4) return 2;
    const int64_t N = atoll(argv[1]);
    const int T = atoi(argv[2]);
    const int64_t tick = atoll(argv[3]);
    std::ios::sync_with_stdio(true);
    T3PluginManager pm;
    // the class schema (Struct XML for NFCClassModule): IObject and Player
    auto prop = [](const char* id, const char* type, bool pub, bool priv) {
        return std::string("<Property Id=\"") + id + "\" Type=\"" + type + "\" Public=\"" + (pub ? "1" : "0") +
               "\" Private=\"" + (priv ? "1" : "0") + "\" Save=\"0\" Cache=\"0\" Ref=\"0\" Upload=\"0\"/>";
    };
    pm.files["NFDataCfg/Struct/LogicClass.xml"] =
        "<XML><Class Id=\"IObject\" Type=\"TYPE_IOBJECT\" Path=\"NFDataCfg/Struct/Class/IObject.xml\" InstancePath=\"\">"
        "<Class Id=\"Player\" Type=\"TYPE_PLAYER\" Path=\"NFDataCfg/Struct/Class/Player.xml\" InstancePath=\"\"/></Class></XML>";
    pm.files["NFDataCfg/Struct/Class/IObject.xml"] =
        "<XML><Propertys>" + prop("ClassName", "string", false, false) + prop("ConfigID", "string", false, false) +
        "</Propertys></XML>";
    pm.files["NFDataCfg/Struct/Class/Player.xml"] =
        "<XML><Propertys>" + prop("SceneID", "int", false, true) + prop("GroupID", "int", false, true) +
        prop("X", "float", true, true) + prop("Y", "float", true, true) + prop("Z", "float", true, true) +
        prop("Level", "int", true, true) + "</Propertys><Records></Records></XML>";
    TestLogModule log;
    pm.AddModule("NFILogModule", &log);
    // the plugins (CREATE_PLUGIN: constructed and Registered), then each one's Install (REGISTER_MODULE)
#ifdef T3_REF
    NFIPlugin* kernel_plugin = new NFKernelPlugin(&pm);
#else
    NFIPlugin* kernel_plugin = new NFGPUKernelPlugin(&pm);
#endif
    for (NFIPlugin* p : {(NFIPlugin*)new NFConfigPlugin(&pm), kernel_plugin, (NFIPlugin*)new Tutorial3Plugin(&pm)}) {
        pm.Registered(p);
        p->Install();
    }
    NFIKernelModule* km = pm.FindModule<NFIKernelModule>();
    NFIEventModule* em = pm.FindModule<NFIEventModule>();
#ifndef T3_REF
    NFGPUKernelAdapter* gk = dynamic_cast<NFGPUKernelAdapter*>(km);
    gk->gpu_.AddHeartBeatProgram("OnHeartBeat", {}, {}, {});  // functor-only: an empty device program
#endif
    auto each = [&](bool (NFIModule::*f)()) {
        for (auto& kv : pm.plugins) (kv.second->*f)();
    };
    g_now = 1700000000000;
    each(&NFIModule::Awake);
    each(&NFIModule::Init);
    each(&NFIModule::AfterInit);  // (Tutorial3's AfterInit: scene 1, its object, DoEvent)
    each(&NFIModule::CheckConfig);
    each(&NFIModule::ReadyExecute);
    std::cout << "== setup done" << std::endl;
    const int spread = (int)std::max<int64_t>(1, 5000 / tick);  // creation windows over the first 5 s
    uint64_t rng = 88172645463325252ull;
    auto next = [&] {
        rng ^= rng << 13;
        rng ^= rng >> 7;
        rng ^= rng << 17;
        return rng;
    };
    int64_t created = 0;
    for (int t = 0; t < T; t++) {
        std::cout << "== frame " << t << std::endl;
        g_now += tick / 2;  // the window, between the frames
        const int64_t upto = t < spread ? N * (t + 1) / spread : N;
        for (; created < upto; created++)  // Player objects in scene 1, group 0 (the tutorial's own object's)
            if (!km->CreateObject(NFGUID(0, 1000 + created), 1, 0, NFrame::Player::ThisName(), "", NFCDataList())) return 3;
        for (int64_t i = 0, k = created / 100; i < k; i++) {  // 1 % of them: DoEvent(1) -> the tutorial's OnEvent
            const int64_t o = (int64_t)(next() % (uint64_t)created);
            em->DoEvent(NFGUID(0, 1000 + o), NFEventDefine(1), NFCDataList() << (NFINT64)(t * 1000 + o) << ("e" + std::to_string(t)));
        }
        g_now += tick - tick / 2;
        each(&NFIModule::Execute);
    }
    std::cout << "== done" << std::endl;
    std::cout.flush();
    _exit(log.errors > 1000000 ? 4 : 0);  // (static destructors: see logic_session.cpp)
}
