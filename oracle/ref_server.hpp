// ref_server.hpp — the parts of a NoahGameFrame server a test program needs around the reference's
// own modules (compiled from /root/reference where they lie): a plugin manager (module registry,
// clock, in-memory config files), a log module, and the workload's class schema written as the
// reference's Struct XML for NFCClassModule.  TEST INFRASTRUCTURE: used by oracle/ref_session.cpp
// (the reference's frame on the CPU) and tests/cpp/adapter_session.cpp (the reference-side plugin).
#pragma once
#include <cstdint>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "NFComm/NFPluginModule/NFILogModule.h"
#include "NFComm/NFPluginModule/NFIPluginManager.h"
#include "../include/nfgpu.h"
#include "nfio.h"

static int64_t g_now = 0;  // the session clock (ms): workload call and frame times

class TestPluginManager : public NFIPluginManager {
public:
    std::map<std::string, NFIModule*> mods;
    std::map<std::string, std::string> files;
    bool ReLoadPlugin(const std::string&) override { return false; }
    void Registered(NFIPlugin*) override {}
    void UnRegistered(NFIPlugin*) override {}
    NFIPlugin* FindPlugin(const std::string&) override { return nullptr; }
    void AddModule(const std::string& n, NFIModule* m) override { mods[n] = m; }
    void RemoveModule(const std::string& n) override { mods.erase(n); }
    NFIModule* FindModule(const std::string& n) override {
        auto it = mods.find(n);
        return it == mods.end() ? nullptr : it->second;
    }
    int GetAppID() const override { return 6; }
    void SetAppID(const int) override {}
    NFINT64 GetInitTime() const override { return 0; }
    NFINT64 GetNowTime() const override { return g_now / 1000; }
    const std::string& GetConfigPath() const override { return path_; }
    void SetConfigName(const std::string&) override {}
    const std::string& GetAppName() const override { return name_; }
    void SetAppName(const std::string&) override {}
    const std::string& GetLogConfigName() const override { return name_; }
    void SetLogConfigName(const std::string&) override {}
    void SetGetFileContentFunctor(GET_FILECONTENT_FUNCTOR) override {}
    bool GetFileContent(const std::string& f, std::string& c) override {
        auto it = files.find(f);
        if (it == files.end()) return false;
        c = it->second;
        return true;
    }

private:
    std::string path_, name_ = "adapter_session";
};

class TestLogModule : public NFILogModule {
public:
    int errors = 0;
    bool LogElement(const NF_LOG_LEVEL l, const NFGUID, const std::string&, const std::string&, const char*, int) override { return note(l); }
    bool LogProperty(const NF_LOG_LEVEL l, const NFGUID, const std::string&, const std::string&, const char*, int) override { return note(l); }
    bool LogObject(const NF_LOG_LEVEL l, const NFGUID, const std::string&, const char*, int) override { return note(l); }
    bool LogRecord(const NF_LOG_LEVEL l, const NFGUID, const std::string&, const std::string&, const int, const int, const char*, int) override { return note(l); }
    bool LogRecord(const NF_LOG_LEVEL l, const NFGUID, const std::string&, const std::string&, const char*, int) override { return note(l); }
    bool LogNormal(const NF_LOG_LEVEL l, const NFGUID, const std::string&, const int, const char*, int) override { return note(l); }
    bool LogNormal(const NF_LOG_LEVEL l, const NFGUID, const std::string&, const std::string&, const char*, int) override { return note(l); }
    bool LogNormal(const NF_LOG_LEVEL l, const NFGUID, const std::ostringstream&, const char*, int) override { return note(l); }

private:
    bool note(NF_LOG_LEVEL l) {
        errors += l >= NLL_ERROR_NORMAL;
        return true;
    }
};

// The workload's classes (NPC, Player) as LogicClass.xml + one file per class: every int / float /
// object property with its Public / Private / Upload flags, every record with its column types
// (tags c0, c1, ...) and flags.
inline void write_class_schema(TestPluginManager& pm, nfio_file& wf, const std::vector<std::string>& pname,
                               const std::vector<std::string>& cname, int64_t NI, int64_t NF, int64_t NC, int64_t NR) {
    const int64_t NP = (int64_t)pname.size();
    const uint8_t* pflags = (const uint8_t*)nfio_get(&wf, "prop_flags")->data;
    auto prop = [](const std::string& id, const char* type, uint8_t f) {
        return "<Property Id=\"" + id + "\" Type=\"" + type + "\" Public=\"" + ((f & NFK_PUBLIC) ? "1" : "0") +
               "\" Private=\"" + ((f & NFK_PRIVATE) ? "1" : "0") + "\" Save=\"0\" Cache=\"0\" Ref=\"0\" Upload=\"" +
               ((f & NFK_UPLOAD) ? "1" : "0") + "\"/>";
    };
    std::string logic = "<XML><Class Id=\"IObject\" Type=\"TYPE_IOBJECT\" Path=\"NFDataCfg/Struct/Class/IObject.xml\" InstancePath=\"\">";
    for (int c = 0; c < NC; c++)  // (the workload's classes only: NPC, then Player)
        logic += "<Class Id=\"" + cname[c] + "\" Type=\"TYPE_" + (c ? "PLAYER" : "NPC") + "\" Path=\"NFDataCfg/Struct/Class/" +
                 cname[c] + ".xml\" InstancePath=\"\"/>";
    pm.files["NFDataCfg/Struct/LogicClass.xml"] = logic + "</Class></XML>";
    pm.files["NFDataCfg/Struct/Class/IObject.xml"] =
        "<XML><Propertys>" + prop("ClassName", "string", 0) + prop("ConfigID", "string", 0) + "</Propertys></XML>";
    for (int c = 0; c < NC; c++) {
        std::string x = "<XML><Propertys>";
        for (int p = 0; p < NP; p++)
            x += prop(pname[p], p < NI ? "int" : p < NI + NF ? "float" : "object", pflags[c * NP + p]);
        x += "</Propertys><Records>";
        for (int r = 0; r < NR; r++) {
            const int32_t rows = ((int32_t*)nfio_get(&wf, "rec_rows")->data)[r];
            const int32_t cols = ((int32_t*)nfio_get(&wf, "rec_cols")->data)[r];
            const uint8_t f = ((uint8_t*)nfio_get(&wf, "rec_flags")->data)[c * NR + r];
            const uint8_t* ct = (const uint8_t*)nfio_get(&wf, "rec_ctype")->data;
            x += "<Record Id=\"rec" + std::to_string(r) + "\" Row=\"" + std::to_string(rows) + "\" Col=\"" +
                 std::to_string(cols) + "\" Public=\"" + ((f & NFK_PUBLIC) ? "1" : "0") + "\" Private=\"" +
                 ((f & NFK_PRIVATE) ? "1" : "0") + "\" Save=\"0\" Cache=\"0\" Upload=\"" + ((f & NFK_UPLOAD) ? "1" : "0") + "\">";
            for (int k = 0; k < cols; k++)
                x += std::string("<Col Type=\"") + (ct[r * NFK_MAX_REC_COLS + k] ? "float" : "int") + "\" Tag=\"c" +
                     std::to_string(k) + "\"/>";
            x += "</Record>";
        }
        x += "</Records></XML>";
        pm.files["NFDataCfg/Struct/Class/" + cname[c] + ".xml"] = x;
    }
}
