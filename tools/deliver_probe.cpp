// deliver_probe.cpp — CPU probe of the plugin's per-call event delivery (NFGPUKernelModule::
// DeliverEvents) on a synthetic frame shaped like config[1]'s: 4096 groups x 256 slots, 8 players
// per group, ~2.3 property events per entity in slot order, public runs of the group's players (but
// the player itself).  Times the loop with the plugin's types and variants of it, to see what the
// per-event cost is made of.  Not part of the product; build: g++ -O2 -std=c++17 -Iinclude.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <vector>

#include "NFGPUKernelModule.hpp"

using namespace nfgpu;

int main(int argc, char** argv) {
    const int G = 4096, S = 256, P = 8;
    const int64_t N = (int64_t)G * S;
    std::mt19937_64 rng(7);
    std::vector<NFGUID> guids(N);
    for (int64_t i = 0; i < N; i++) guids[i] = NFGUID(1 + (int64_t)(rng() % 4), (int64_t)rng());
    std::vector<int32_t> ev_obj, ev_pid;
    std::vector<uint64_t> ev_old, ev_new;
    std::vector<uint32_t> msg_off{0}, msg_rcpt;
    for (int g = 0; g < G; g++) {
        for (int s = 0; s < S; s++) {
            const int64_t o = (int64_t)g * S + s;
            const bool player = s % (S / P) == 0;
            const int ne = (int)(rng() % 5);  // 0..4 events, mean 2
            for (int k = 0; k < ne; k++) {
                ev_obj.push_back((int32_t)o);
                ev_pid.push_back((int32_t)(rng() % 10));
                ev_old.push_back(rng());
                ev_new.push_back(rng());
                for (int q = 0; q < P; q++) {
                    const int64_t r = (int64_t)g * S + q * (S / P);
                    if (player && r == o) continue;
                    msg_rcpt.push_back((uint32_t)r);
                }
                msg_off.push_back((uint32_t)msg_rcpt.size());
            }
        }
    }
    const int64_t ne = (int64_t)ev_obj.size();
    std::vector<NFGUID> ev_self(ne);
    for (int64_t e = 0; e < ne; e++) ev_self[e] = guids[ev_obj[e]];
    std::vector<uint8_t> ev_same(ne);
    for (int64_t e = 1; e < ne; e++)
        ev_same[e] = msg_off[e + 1] - msg_off[e] == msg_off[e] - msg_off[e - 1] &&
                     !memcmp(&msg_rcpt[msg_off[e]], &msg_rcpt[msg_off[e - 1]], 4 * (msg_off[e + 1] - msg_off[e]));
    struct PD { std::string name; TDATA_TYPE type; };
    std::vector<PD> props(10);
    for (int i = 0; i < 10; i++) props[i] = {"Prop" + std::to_string(i), i < 7 ? TDATA_INT : TDATA_FLOAT};
    std::vector<int> def_of(10);
    for (int i = 0; i < 10; i++) def_of[i] = i;
    int64_t n_prop = 0, n_rcpt = 0;
    std::vector<PROPERTY_EVENT_FUNCTOR> common{[&](const NFGUID&, const std::string&, const TData&, const TData&) {
        n_prop++;
        return 0;
    }};
    std::vector<PROPERTY_SINGLE_EVENT_FUNCTOR> aoi{[&](const NFGUID&, const std::string&, const TData&, const TData&,
                                                       const std::vector<NFGUID>& to) {
        n_rcpt += (int64_t)to.size();
        return 0;
    }};
    int64_t rebuilds = 0;
    auto run = [&](int variant) {
        std::vector<NFGUID> rcpt;
        TData a, b;
        for (int64_t e = 0; e < ne; e++) {
            const PD& pd = props[variant == 7 ? 0 : def_of[ev_pid[e]]];
            if (variant == 8 || variant == 9) {  // fresh per-event values, built in registers
                const bool isi = pd.type == TDATA_INT, isf = pd.type == TDATA_FLOAT;
                TData x, y;
                x.type = y.type = pd.type;
                const uint64_t vo = ev_old[e], vn = ev_new[e];
                const uint64_t mi = isi ? ~0ull : 0ull, mf = isf ? ~0ull : 0ull;  // (branch-free)
                x.i = (int64_t)(vo & mi);
                y.i = (int64_t)(vn & mi);
                const uint64_t fo = vo & mf, fn = vn & mf;
                memcpy(&x.f, &fo, 8);
                memcpy(&y.f, &fn, 8);
                const NFGUID& self = ev_self[e];
                if (variant == 8) {
                    n_prop += x.i ^ y.i ^ self.nData64;
                    continue;
                }
                for (auto& cb : common) cb(self, pd.name, x, y);
                if (msg_off[e + 1] > msg_off[e]) {
                    const uint32_t m0 = msg_off[e], m1 = msg_off[e + 1];
                    if (!ev_same[e]) {
                        rebuilds++;
                        rcpt.resize(m1 - m0);
                        for (uint32_t m = m0; m < m1; m++) rcpt[m - m0] = guids[msg_rcpt[m]];
                    }
                    for (auto& cb : aoi) cb(self, pd.name, x, y, rcpt);
                }
                continue;
            }
            if (variant == 6) {  // every field written once, with its final value
                const bool isi = pd.type == TDATA_INT, isf = pd.type == TDATA_FLOAT;
                double fo, fn;
                memcpy(&fo, &ev_old[e], 8);
                memcpy(&fn, &ev_new[e], 8);
                a.type = b.type = pd.type;
                a.i = isi ? (int64_t)ev_old[e] : 0;
                b.i = isi ? (int64_t)ev_new[e] : 0;
                a.f = isf ? fo : 0.0;
                b.f = isf ? fn : 0.0;
                a.o = b.o = NFGUID();
                n_prop += a.i ^ b.i ^ ev_self[e].nData64;
                continue;
            } else {
                a = b = TData{};
            }
            a.type = b.type = pd.type;
            if (variant >= 5) {  // branch-free: both views written, the type says which is read
                a.i = (int64_t)ev_old[e];
                b.i = (int64_t)ev_new[e];
                memcpy(&a.f, &ev_old[e], 8);
                memcpy(&b.f, &ev_new[e], 8);
            } else if (pd.type == TDATA_INT) {
                a.i = (int64_t)ev_old[e];
                b.i = (int64_t)ev_new[e];
            } else {
                memcpy(&a.f, &ev_old[e], 8);
                memcpy(&b.f, &ev_new[e], 8);
            }
            const NFGUID& self = ev_self[e];
            if (variant == 3 || variant >= 5) {
                n_prop += a.i ^ b.i ^ self.nData64;
                continue;
            }
            if (variant != 1 && variant != 4)
                for (auto& cb : common) cb(self, pd.name, a, b);
            if (msg_off[e + 1] > msg_off[e]) {
                const uint32_t m0 = msg_off[e], m1 = msg_off[e + 1];
                if (!ev_same[e]) {
                    rebuilds++;
                    rcpt.resize(m1 - m0);
                    for (uint32_t m = m0; m < m1; m++) rcpt[m - m0] = guids[msg_rcpt[m]];
                }
                if (variant != 2 && variant != 4)
                    for (auto& cb : aoi) cb(self, pd.name, a, b, rcpt);
            }
        }
    };
    {
        for (int rep = 0; rep < 3; rep++) {
            const auto t0 = std::chrono::steady_clock::now();
            uint64_t x = 0;
            for (int64_t e = 0; e < ne; e++) x += ev_old[e] ^ ev_new[e] ^ (uint64_t)ev_pid[e] ^ (uint64_t)ev_self[e].nData64;
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            printf("stream sum     %8.2f ms  %6.2f ns/event (%llu)\n", ms, ms * 1e6 / ne, (unsigned long long)x);
        }
    }
    const char* names[] = {"full", "no common cb", "no aoi cb", "reads only", "no cbs", "reads brfree", "reads nozero", "reads noprop", "fresh reads", "fresh full"};
    for (int rep = 0; rep < 2; rep++)
        for (int v = 0; v < 10; v++) {
            rebuilds = 0;
            const auto t0 = std::chrono::steady_clock::now();
            run(v);
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            printf("%-14s %8.2f ms  %6.2f ns/event  events %lld msgs %zu rebuilds %lld\n", names[v], ms, ms * 1e6 / ne,
                   (long long)ne, msg_rcpt.size(), (long long)rebuilds);
        }
    {  // the heartbeat functor walk (gathered: dense entries, NFGUIDs, intervals; pool in walk order)
        const int64_t nf = N * 13 / 10;
        std::vector<OBJECT_SCHEDULE_FUNCTOR> pool(nf);
        int64_t n_hb = 0;
        OBJECT_SCHEDULE_FUNCTOR hb = [&](const NFGUID&, const std::string&, const float, const int) {
            n_hb++;
            return 0;
        };
        for (auto& x : pool) x = hb;
        std::vector<int32_t> fc(nf), fk(nf), fr(nf);
        std::vector<NFGUID> fg(nf);
        std::vector<float> ft(nf);
        for (int64_t i = 0; i < nf; i++) {
            fc[i] = (int32_t)i;
            fk[i] = (int32_t)(rng() % 5);
            fr[i] = (int32_t)(rng() % 10);
            fg[i] = guids[i % N];
            ft[i] = 0.1f;
        }
        std::vector<std::string> kn{"HPRegen", "MPRegen", "Move", "Patrol", "Poison"};
        for (int rep = 0; rep < 3; rep++) {
            const auto t0 = std::chrono::steady_clock::now();
            for (int64_t i = 0; i < nf; i++) {
                const int32_t c = fc[i];
                if (c >= 0 && pool[c]) pool[c](fg[i], kn[fk[i]], ft[i], fr[i]);
            }
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            printf("functor walk   %8.2f ms  %6.2f ns/call (%lld)\n", ms, ms * 1e6 / nf, (long long)n_hb);
        }
        struct FE { const OBJECT_SCHEDULE_FUNCTOR* fn; const std::string* name; NFGUID g; float t; int32_t r; };
        std::vector<FE> fe(nf);
        for (int64_t i = 0; i < nf; i++) fe[i] = {&pool[fc[i]], &kn[fk[i]], fg[i], ft[i], fr[i]};
        for (int rep = 0; rep < 3; rep++) {
            const auto t0 = std::chrono::steady_clock::now();
            for (int64_t i = 0; i < nf; i++) {
                const FE& x = fe[i];
                (*x.fn)(x.g, *x.name, x.t, x.r);
            }
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            printf("functor AoS    %8.2f ms  %6.2f ns/call (%lld)\n", ms, ms * 1e6 / nf, (long long)n_hb);
        }
    }
    printf("(%lld %lld)\n", (long long)n_prop, (long long)n_rcpt);
    (void)argc;
    (void)argv;
    return 0;
}
