// module_sched.cpp — NFIScheduleModule module schedules through nfgpu::ModuleScheduler (the plugin's
// host-side restatement of NFCScheduleModule, SM:123-216), driven by a script; prints what the
// functors see so tests/test_boundary.py can diff it against the reference's NFCScheduleModule
// (oracle/_ref/nf_ref_harness --module-script, same script).  CPU only.
//
// script lines: <now_ms> add <name> <fTime> <count> | <now_ms> remove <name> | <now_ms> exec |
//               <now_ms> exist <name>
#include <cstdio>
#include <string>

#include "NFGPUKernelModule.hpp"

int main(int argc, char** argv) {
    if (argc != 2) return 2;
    FILE* f = fopen(argv[1], "r");
    if (!f) return 2;
    nfgpu::ModuleScheduler ms;
    int64_t now = 0;
    auto clock = [&] { return now; };
    auto cb = [&](const std::string& name, const float t, const int remain) {
        printf("fire %lld %s %.3f %d\n", (long long)now, name.c_str(), t, remain);
        return 0;
    };
    char op[16], name[64];
    long long t;
    while (fscanf(f, "%lld %15s", &t, op) == 2) {
        now = t;
        std::string o(op);
        if (o == "add") {
            float ft;
            int cnt;
            if (fscanf(f, "%63s %f %d", name, &ft, &cnt) != 3) return 3;
            ms.AddSchedule(name, cb, ft, cnt, now);
        } else if (o == "remove") {
            if (fscanf(f, "%63s", name) != 1) return 3;
            ms.RemoveSchedule(name);
        } else if (o == "exist") {
            if (fscanf(f, "%63s", name) != 1) return 3;
            printf("exist %lld %s %d\n", (long long)now, name, ms.ExistSchedule(name) ? 1 : 0);
        } else if (o == "exec") {
            ms.Execute(clock);
        } else {
            return 3;
        }
    }
    fclose(f);
    return 0;
}
