// jmap_check.cpp — TEST INFRASTRUCTURE: differential check of the product's
// HashMap-order model (siddhi_amd/csrc/sh_jmap.h) against the oracle's
// restatement of java.util.HashMap (oracle/jhashmap.h) on random operation
// sequences: computeIfAbsent of new and present keys, iterator removal
// (movable = false) and HashMap.remove (movable = true), with key sets that
// collide on purpose (equal String.hashCode) so bins treeify, split and shrink.
// Prints the first diverging step, exits 1 on divergence.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../oracle/jhashmap.h"
#include "../../siddhi_amd/csrc/sh_jmap.h"

static std::vector<std::u16string> g_keys;

static std::u16string make_key(std::mt19937_64& rng, int mode, int i) {
    std::string s;
    if (mode == 0) {
        s = "user" + std::to_string(i);
    } else if (mode == 1) {
        // "Aa" and "BB" share String.hashCode: blocks of them collide fully
        const int len = 3 + (int)(rng() % 3);
        for (int b = 0; b < len; b++) s += (rng() & 1) ? "Aa" : "BB";
        s += std::to_string(i % 7);
    } else {
        const int len = 1 + (int)(rng() % 6);
        for (int b = 0; b < len; b++) s += (char)('a' + rng() % 26);
    }
    return std::u16string(s.begin(), s.end());
}

int main(int argc, char** argv) {
    const int seeds = argc > 1 ? atoi(argv[1]) : 200;
    int bad = 0;
    for (int seed = 0; seed < seeds && !bad; seed++) {
        std::mt19937_64 rng(seed * 7919 + 13);
        const int mode = seed % 3;
        const int nk = 50 + (int)(rng() % 3000);
        g_keys.clear();
        for (int i = 0; i < nk; i++) g_keys.push_back(make_key(rng, mode, i));
        auto cmp = [](int64_t a, int64_t b) {
            return ref::java_string_compare((const uint16_t*)g_keys[a].data(), (int64_t)g_keys[a].size(),
                                            (const uint16_t*)g_keys[b].data(), (int64_t)g_keys[b].size());
        };
        auto hsh = [](int64_t k) {
            return ref::java_string_hash((const uint16_t*)g_keys[k].data(), (int64_t)g_keys[k].size());
        };
        ref::JHashMap O;
        O.compare = cmp;
        O.string_hash = hsh;
        ShJMap P;
        P.cmp = [&](int32_t a, int32_t b) { return cmp(a, b); };
        const int steps = 4000 + (int)(rng() % 8000);
        for (int st = 0; st < steps; st++) {
            const int op = (int)(rng() % 10);
            const int32_t k = (int32_t)(rng() % nk);
            if (op < 6) {
                O.computeIfAbsent(k);
                P.set_hash(k, hsh(k));
                P.compute_if_absent(k);
            } else if (op < 9) {
                // returnAllStates: remove a batch of present keys in iteration order
                std::vector<int64_t> order = O.keys();
                std::vector<int32_t> rm;
                for (int64_t x : order)
                    if (rng() % 4 == 0) rm.push_back((int32_t)x);
                std::vector<int32_t> rm2 = rm;
                P.sort_iteration(rm2);
                if (rm2 != rm) {
                    printf("seed %d step %d: removal order differs\n", seed, st);
                    bad = 1;
                    break;
                }
                for (int32_t x : rm) {
                    O.remove(x, false);
                    P.remove(x, false);
                }
            } else {
                if (O.contains(k)) {
                    O.remove(k, true);
                    P.remove(k, true);
                }
            }
            // iteration order == rank order
            std::vector<int64_t> a = O.keys();
            std::vector<std::pair<uint64_t, int32_t>> r;
            for (int64_t x : a) {
                if (!P.present((int32_t)x)) {
                    printf("seed %d step %d: key %lld missing in the model\n", seed, st, (long long)x);
                    bad = 1;
                    break;
                }
                r.push_back({P.rank((int32_t)x), (int32_t)x});
            }
            if (bad) break;
            if ((int)a.size() != P.size || O.capacity() != P.cap()) {
                printf("seed %d step %d: size %zu/%d cap %d/%d\n", seed, st, a.size(), P.size, O.capacity(), P.cap());
                bad = 1;
                break;
            }
            for (size_t i = 1; i < r.size(); i++)
                if (!(r[i - 1].first < r[i].first)) {
                    printf("seed %d step %d: rank order differs at %zu (keys %d %d, bins %llu %llu)\n", seed, st, i,
                           r[i - 1].second, r[i].second, (unsigned long long)(r[i - 1].first >> 38),
                           (unsigned long long)(r[i].first >> 38));
                    bad = 1;
                    break;
                }
            if (bad) break;
            P.dirty.clear();
        }
    }
    if (!bad) printf("ok: %d seeds\n", seeds);
    return bad;
}
