// NFGPUKernelPlugin.cpp — the REFERENCE-SIDE plugin a NoahGameFrame maintainer adds to swap the
// MI355X frame path in for NFKernelPlugin.  It compiles against the
// reference's own headers (tests/test_boundary.py::test_integration_adapter_compiles checks it
// with `g++ -fsyntax-only -I<reference> -I<reference>/Dependencies -Iinclude`), and links against
// libnfgpu_plugin.so / libnfgpu.so plus the reference's NFCore and NFKernelPlugin objects.
//
//   NFGPUKernelAdapter    NFIKernelModule (NFIKernelModule.h:103-148): the frame-path calls go to
//                         nfgpu::NFGPUKernelModule; everything else (string / object properties,
//                         object lists, class events) stays in the reference's NFCKernelModule.
//   NFGPUScheduleAdapter  NFIScheduleModule (NFIScheduleModule.h:23-39): every pure virtual, object
//                         schedules on the device, module schedules on the host.
//   NFGPUKernelPlugin     the NFIPlugin that registers both (NFKernelPlugin.cpp:40-46 pattern).
#include <memory>
#include <string>
#include <vector>

#include "NFComm/NFKernelPlugin/NFCEventModule.h"
#include "NFComm/NFKernelPlugin/NFCKernelModule.h"
#include "NFComm/NFKernelPlugin/NFCSceneAOIModule.h"
#include "NFComm/NFPluginModule/NFIPlugin.h"
#include "NFComm/NFPluginModule/NFIPluginManager.h"
#include "NFComm/NFPluginModule/NFIScheduleModule.h"
#include "NFComm/NFPluginModule/NFPlatform.h"
#include "NFGPUKernelModule.hpp"

namespace {
nfgpu::NFGUID to_gpu(const NFGUID& g) { return nfgpu::NFGUID(g.nHead64, g.nData64); }
NFGUID to_ref(const nfgpu::NFGUID& g) { return NFGUID(g.nHead64, g.nData64); }
}  // namespace

class NFGPUKernelAdapter : public NFCKernelModule {
public:
    explicit NFGPUKernelAdapter(NFIPluginManager* p) : NFCKernelModule(p), gpu_(/*capacity=*/1 << 20) {
        gpu_.SetTimeSource([] { return NFGetTime(); });  // NFPlatform.h:367, as NFCScheduleModule reads it
    }
    bool AfterInit() override {
        NFCKernelModule::AfterInit();
        // schema: one gpu_.AddProperty per int / float property of Struct/Class/*.xml, one
        // SetPropertyFlags(class, property, Public, Private, Upload) per class, one
        // AddHeartBeatProgram(name, ops) per schedule name the game logic uses (no ops for a
        // functor-only heartbeat), then the objects created so far: gpu_.CreateObject(...)
        return gpu_.AfterInit();
    }
    bool Execute() override {  // NFCKernelModule::Execute (KM:70) + NFCScheduleModule::Execute (SM:49) + AOI fan-out
        NFCKernelModule::Execute();
        return gpu_.Execute();
    }
    bool SetPropertyInt(const NFGUID& self, const std::string& name, const NFINT64 v) override {  // KM:323
        return gpu_.SetPropertyInt(to_gpu(self), name, v);
    }
    bool SetPropertyFloat(const NFGUID& self, const std::string& name, const double v) override {  // KM:336
        return gpu_.SetPropertyFloat(to_gpu(self), name, v);
    }
    NFINT64 GetPropertyInt(const NFGUID& self, const std::string& name) override {  // KM:401, read-your-writes
        return gpu_.GetPropertyInt(to_gpu(self), name);
    }
    double GetPropertyFloat(const NFGUID& self, const std::string& name) override {  // KM:413
        return gpu_.GetPropertyFloat(to_gpu(self), name);
    }
    bool SetRecordInt(const NFGUID& self, const std::string& rec, const int nRow, const int nCol,
                      const NFINT64 v) override {  // KM:505
        return gpu_.SetRecordInt(to_gpu(self), rec, nRow, nCol, v);
    }
    bool SetRecordFloat(const NFGUID& self, const std::string& rec, const int nRow, const int nCol,
                        const double v) override {  // KM:545
        return gpu_.SetRecordFloat(to_gpu(self), rec, nRow, nCol, v);
    }
    NFINT64 GetRecordInt(const NFGUID& self, const std::string& rec, const int nRow, const int nCol) override {
        return gpu_.GetRecordInt(to_gpu(self), rec, nRow, nCol);  // NFIKernelModule.h:134, read-your-writes
    }
    double GetRecordFloat(const NFGUID& self, const std::string& rec, const int nRow, const int nCol) override {
        return gpu_.GetRecordFloat(to_gpu(self), rec, nRow, nCol);  // NFIKernelModule.h:135
    }
    bool SwitchScene(const NFGUID& self, const int scene, const int group, const float fX, const float fY,
                     const float fZ, const float fOrient, const NFIDataList& arg) override {  // NFIKernelModule.h:148
        NFCKernelModule::SwitchScene(self, scene, group, fX, fY, fZ, fOrient, arg);  // host-side scene lists
        return gpu_.SwitchScene(to_gpu(self), scene, group, fX, fY, fZ, fOrient);
    }
    bool DestroyObject(const NFGUID& self) override {  // KM:273
        // the reference's DestroyObject reads SceneID / GroupID through GetPropertyInt (KM:283-284),
        // which this adapter answers from the device: it runs while the object is still there
        const bool ok = NFCKernelModule::DestroyObject(self);
        gpu_.DestroyObject(to_gpu(self));
        return ok;
    }
    nfgpu::NFGPUKernelModule gpu_;
};

class NFGPUScheduleAdapter : public NFIScheduleModule {
public:
    explicit NFGPUScheduleAdapter(NFIPluginManager* p) { pPluginManager = p; }

    // ---- module schedules (NFIScheduleModule.h:23-25) ----
    bool AddSchedule(const std::string& name, const MODULE_SCHEDULE_FUNCTOR_PTR& cb, const float fTime,
                     const int nCount) override {
        return gpu().AddSchedule(name,
                                 [cb](const std::string& n, const float t, const int c) { return (*cb)(n, t, c); },
                                 fTime, nCount);
    }
    bool RemoveSchedule(const std::string& name) override { return gpu().RemoveSchedule(name); }
    bool ExistSchedule(const std::string& name) override { return gpu().ExistSchedule(name); }

    // ---- object schedules (NFIScheduleModule.h:36-39) ----
    bool AddSchedule(const NFGUID self, const std::string& name, const OBJECT_SCHEDULE_FUNCTOR_PTR& cb,
                     const float fTime, const int nCount) override {  // SM:257
        return gpu().AddSchedule(
            to_gpu(self), name,
            [cb](const nfgpu::NFGUID& g, const std::string& n, const float t, const int c) { return (*cb)(to_ref(g), n, t, c); },
            fTime, nCount);
    }
    bool RemoveSchedule(const NFGUID self) override { return gpu().RemoveSchedule(to_gpu(self)); }  // SM:240
    bool RemoveSchedule(const NFGUID self, const std::string& name) override {                       // SM:245
        return gpu().RemoveSchedule(to_gpu(self), name);
    }
    bool ExistSchedule(const NFGUID self, const std::string& name) override {  // SM:276
        return gpu().ExistSchedule(to_gpu(self), name);
    }
    // the frame (object and module schedules) runs in NFGPUKernelAdapter::Execute
    bool Execute() override { return true; }

private:
    nfgpu::NFGPUKernelModule& gpu() {
        return dynamic_cast<NFGPUKernelAdapter*>(pPluginManager->FindModule<NFIKernelModule>())->gpu_;
    }
};

class NFGPUKernelPlugin : public NFIPlugin {
public:
    explicit NFGPUKernelPlugin(NFIPluginManager* p) { pPluginManager = p; }
    const int GetPluginVersion() override { return 0; }
    const std::string GetPluginName() override { return GET_CLASS_NAME(NFGPUKernelPlugin); }
    void Install() override {
        REGISTER_MODULE(pPluginManager, NFISceneAOIModule, NFCSceneAOIModule)  // non-frame AOI (enter / leave)
        REGISTER_MODULE(pPluginManager, NFIKernelModule, NFGPUKernelAdapter)
        REGISTER_MODULE(pPluginManager, NFIEventModule, NFCEventModule)
        REGISTER_MODULE(pPluginManager, NFIScheduleModule, NFGPUScheduleAdapter)
    }
    void Uninstall() override {
        UNREGISTER_MODULE(pPluginManager, NFIScheduleModule, NFGPUScheduleAdapter)
        UNREGISTER_MODULE(pPluginManager, NFIEventModule, NFCEventModule)
        UNREGISTER_MODULE(pPluginManager, NFIKernelModule, NFGPUKernelAdapter)
        UNREGISTER_MODULE(pPluginManager, NFISceneAOIModule, NFCSceneAOIModule)
    }
};

#ifdef NF_DYNAMIC_PLUGIN
NF_EXPORT void DllStartPlugin(NFIPluginManager* pm) { CREATE_PLUGIN(pm, NFGPUKernelPlugin) }
NF_EXPORT void DllStopPlugin(NFIPluginManager* pm) { DESTROY_PLUGIN(pm, NFGPUKernelPlugin) }
#endif
