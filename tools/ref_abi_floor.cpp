// ref_abi_floor.cpp — the per-event floor of delivering frame events through the reference's own callback
// ABI (NFIDataList::TData variants, NFCDataList recipient lists, std::function callbacks), no device
// work: what the drop-in adapter's delivery cannot go below.  Built from the reference
// sources where they lie:  g++ -O2 -I$REF -I$REF/Dependencies tools/ref_abi_floor.cpp
// $REF/NFComm/NFCore/NFCDataList.cpp $REF/NFComm/NFCore/NFMemoryCounter.cpp
#include <chrono>
#include <cstdio>
#include <memory>
#include <vector>
#include "NFComm/NFCore/NFCDataList.h"
#include "NFComm/NFPluginModule/NFIKernelModule.h"
int main() {
    const int N = 2400000;
    std::vector<int64_t> vals(N);
    for (int i = 0; i < N; i++) vals[i] = i * 7;
    int64_t sink = 0, rc = 0;
    PROPERTY_EVENT_FUNCTOR_PTR cb(new PROPERTY_EVENT_FUNCTOR([&](const NFGUID& s, const std::string& n, const NFIDataList::TData& a, const NFIDataList::TData& b) { sink += a.GetInt() ^ b.GetInt(); return 0; }));
    typedef std::function<int(const NFGUID&, const std::string&, const NFIDataList::TData&, const NFIDataList::TData&, const NFIDataList&)> AOICB;
    std::shared_ptr<AOICB> aoi(new AOICB([&](const NFGUID&, const std::string&, const NFIDataList::TData&, const NFIDataList::TData&, const NFIDataList& l) { rc += l.GetCount(); return 0; }));
    NFCDataList rl;
    for (int k = 0; k < 8; k++) rl.Add(NFGUID(1, k));
    const std::string name = "HP";
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) {
        NFIDataList::TData ra, rb;
        ra.SetInt(vals[i]);
        rb.SetInt(vals[i] + 1);
        const NFGUID s(1, i);
        (*cb)(s, name, ra, rb);
        (*aoi)(s, name, ra, rb, rl);
        if ((i & 7) == 0) { rl.Clear(); for (int k = 0; k < 8; k++) rl.Add(NFGUID(1, k + i)); }
    }
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("%d events: %.1f ms (%.1f ns/event) sink %lld rc %lld\n", N, ms, ms * 1e6 / N, (long long)sink, (long long)rc);
}
