// sh_jmap.h — iteration order of siddhi-core's scheduler HashMap, host side of
// libsiddhi_hip.so.
//
// Scheduler.onTimeChange (core/util/Scheduler.java:75-87) walks
// PartitionStateHolder.states (a java.util.HashMap<String, ...> keyed by the
// partition key's toString(), util/snapshot/state/PartitionStateHolder.java:36)
// and hands every due SchedulerState to a TreeMultimap whose value comparator is
// always 0 (Scheduler.java:364-366): per distinct due time only the FIRST state
// in HashMap iteration order fires. The device picks that state as the minimum
// of a per-key 64-bit rank = bucket << 38 | position code; this model keeps the
// ranks exact by replaying the map's structural history (OpenJDK 8
// java.util.HashMap): computeIfAbsent with its lazy resize (size > threshold on
// any call) and head insertion, treeifyBin (>= 8 nodes at capacity >= 64, else
// resize), TreeNode insertion after the tree parent + moveRootToFront, split on
// resize (untreeify at <= 6), removeTreeNode, and iterator removal (movable =
// false) from returnAllStates.
//
// Position codes: a plain bin in insertion-head order gets MAXC - insert ordinal
// (a new head sorts first); a bin that ever held a tree ("irregular") gets its
// list positions recomputed on every change. Nodes live in per-key arrays (key
// ids are dense); only the order is modelled, never the values.
#pragma once
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <functional>
#include <unordered_set>
#include <vector>

struct ShJMap {
    static const int kTreeify = 8, kUntreeify = 6, kMinTreeifyCap = 64;
    static const int kMaxCap = 1 << 30;
    static const uint64_t kMaxCode = (1ull << 38) - 1;
    static const int kRankBucketBits = 26;  // rank = bucket << 38 | code

    // per key (dense ids)
    std::vector<int32_t> h;        // spread hash (registered once per key)
    std::vector<int32_t> nx, pv, pa, lf, rt;
    std::vector<uint8_t> fl;       // 1 present, 2 tree node, 4 red
    std::vector<uint64_t> code;
    std::vector<int32_t> tab;      // bin heads, -1 empty
    int32_t size = 0, threshold = 0;
    uint64_t ord = 0;              // insert ordinal (plain-bin codes)
    std::unordered_set<int32_t> irregular;  // bins whose order left insertion-head form
    // String.compareTo of two keys' toString()
    std::function<int(int32_t, int32_t)> cmp;
    // outputs of the last operations: keys whose rank changed, full re-rank needed
    std::vector<int32_t> dirty;
    bool rerank_all = false;

    void ensure(int32_t k) {
        if (k < (int32_t)h.size()) return;
        const size_t n = std::max<size_t>((size_t)k + 1, h.size() * 2);
        h.resize(n, 0);
        nx.resize(n, -1);
        pv.resize(n, -1);
        pa.resize(n, -1);
        lf.resize(n, -1);
        rt.resize(n, -1);
        fl.resize(n, 0);
        code.resize(n, 0);
    }
    static int32_t spread(int32_t x) { return x ^ (int32_t)((uint32_t)x >> 16); }
    void set_hash(int32_t k, int32_t string_hash) {
        ensure(k);
        h[k] = spread(string_hash);
    }
    bool present(int32_t k) const { return k < (int32_t)fl.size() && (fl[k] & 1); }
    bool is_tree(int32_t k) const { return (fl[k] & 2) != 0; }
    bool red(int32_t k) const { return k >= 0 && (fl[k] & 4) != 0; }
    void set_red(int32_t k, bool r) {
        if (r) fl[k] |= 4;
        else fl[k] &= (uint8_t)~4;
    }
    int cap() const { return (int)tab.size(); }
    int bin_of(int32_t k) const { return (cap() - 1) & h[k]; }
    uint64_t rank(int32_t k) const { return ((uint64_t)(uint32_t)bin_of(k) << 38) | code[k]; }
    bool rank_fits() const { return cap() <= (1 << kRankBucketBits); }

    // list positions of an irregular bin become its codes
    void recode_bin(int b) {
        uint64_t pos = 0;
        for (int32_t e = tab[b]; e >= 0; e = nx[e]) {
            code[e] = pos++;
            dirty.push_back(e);
        }
        if (tab[b] < 0) irregular.erase(b);
    }
    void touch_bin(int b) {
        if (irregular.count(b)) recode_bin(b);
    }

    // -------------------------------------------------------------- operations
    // any PartitionStateHolder.getState call: computeIfAbsent(key, ...); true when added
    bool compute_if_absent(int32_t k) {
        ensure(k);
        if (size > threshold || tab.empty()) resize();
        if (present(k)) return false;
        const int i = bin_of(k);
        const int32_t first = tab[i];
        int bin_count = 0;
        const bool tree_bin = first >= 0 && is_tree(first);
        if (!tree_bin)
            for (int32_t e = first; e >= 0; e = nx[e]) ++bin_count;
        fl[k] = 1;
        pa[k] = lf[k] = rt[k] = pv[k] = -1;
        if (tree_bin) {
            put_tree_val(first, k);
            irregular.insert(i);
            recode_bin(i);
        } else {
            nx[k] = first;  // newNode(hash, key, value, first): the new head
            tab[i] = k;
            code[k] = kMaxCode - (ord++ & kMaxCode);
            dirty.push_back(k);
            if (bin_count >= kTreeify - 1) treeify_bin(h[k]);
            touch_bin(bin_of(k));
        }
        ++size;
        return true;
    }
    // a getState of a present key (only its lazy-resize side effect matters)
    void touch() {
        if (size > threshold || tab.empty()) resize();
    }
    // HashMap.removeNode(hash, key, null, false, movable)
    void remove(int32_t k, bool movable) {
        if (!present(k) || tab.empty()) return;
        const int idx = bin_of(k);
        if (is_tree(k)) {
            remove_tree_node(k, movable);
        } else if (tab[idx] == k) {
            tab[idx] = nx[k];
        } else {
            int32_t p = tab[idx];
            while (nx[p] != k) p = nx[p];
            nx[p] = nx[k];
        }
        fl[k] = 0;
        nx[k] = pv[k] = pa[k] = lf[k] = rt[k] = -1;
        --size;
        touch_bin(idx);
    }
    // keys in iteration order among `ks` (returnAllStates removal order)
    void sort_iteration(std::vector<int32_t>& ks) const {
        std::vector<std::pair<uint64_t, int32_t>> r;
        r.reserve(ks.size());
        for (int32_t k : ks) {
            uint64_t pos = 0;
            if (present(k) && irregular.count(bin_of(k))) {
                for (int32_t e = tab[bin_of(k)]; e >= 0 && e != k; e = nx[e]) ++pos;
            } else if (present(k)) {
                pos = code[k];
            }
            r.push_back({((uint64_t)(uint32_t)(present(k) ? bin_of(k) : 0) << 38) | pos, k});
        }
        std::stable_sort(r.begin(), r.end(),
                         [](const std::pair<uint64_t, int32_t>& a, const std::pair<uint64_t, int32_t>& b) {
                             return a.first < b.first;
                         });
        for (size_t i = 0; i < r.size(); i++) ks[i] = r[i].second;
    }

   private:
    void resize() {
        const int old_cap = cap();
        const int old_thr = threshold;
        int new_cap = 0, new_thr = 0;
        if (old_cap > 0) {
            if (old_cap >= kMaxCap) {
                threshold = 0x7FFFFFFF;
                return;
            }
            new_cap = old_cap << 1;
            if (new_cap < kMaxCap && old_cap >= 16) new_thr = old_thr << 1;
        } else if (old_thr > 0) {
            new_cap = old_thr;
        } else {
            new_cap = 16;
            new_thr = 12;
        }
        if (new_thr == 0) {
            const float ft = (float)new_cap * 0.75f;
            new_thr = (new_cap < kMaxCap && ft < (float)kMaxCap) ? (int)ft : 0x7FFFFFFF;
        }
        threshold = new_thr;
        std::vector<int32_t> old;
        old.swap(tab);
        tab.assign(new_cap, -1);
        std::unordered_set<int32_t> old_irr;
        old_irr.swap(irregular);
        rerank_all = true;
        for (int j = 0; j < old_cap; ++j) {
            const int32_t e = old[j];
            if (e < 0) continue;
            const bool irr = old_irr.count(j) != 0;
            if (nx[e] < 0) {
                tab[h[e] & (new_cap - 1)] = e;
                if (irr) mark_irregular(h[e] & (new_cap - 1));
            } else if (is_tree(e)) {
                split(e, j, old_cap);
                mark_irregular(j);
                mark_irregular(j + old_cap);
            } else {
                int32_t lo_h = -1, lo_t = -1, hi_h = -1, hi_t = -1;
                for (int32_t x = e; x >= 0;) {
                    const int32_t n = nx[x];
                    if ((h[x] & old_cap) == 0) {
                        if (lo_t < 0) lo_h = x;
                        else nx[lo_t] = x;
                        lo_t = x;
                    } else {
                        if (hi_t < 0) hi_h = x;
                        else nx[hi_t] = x;
                        hi_t = x;
                    }
                    x = n;
                }
                if (lo_t >= 0) {
                    nx[lo_t] = -1;
                    tab[j] = lo_h;
                }
                if (hi_t >= 0) {
                    nx[hi_t] = -1;
                    tab[j + old_cap] = hi_h;
                }
                if (irr) {
                    mark_irregular(j);
                    mark_irregular(j + old_cap);
                }
            }
        }
    }
    void mark_irregular(int b) {
        if (b < cap() && tab[b] >= 0) {
            irregular.insert(b);
            recode_bin(b);
        }
    }
    void treeify_bin(int32_t hash) {
        if (cap() < kMinTreeifyCap) {
            resize();
            return;
        }
        const int idx = (cap() - 1) & hash;
        int32_t hd = tab[idx];
        if (hd < 0) return;
        int32_t tl = -1;
        for (int32_t e = hd; e >= 0; e = nx[e]) {  // replacementTreeNode: same list order
            fl[e] = (uint8_t)((fl[e] & 1) | 2);
            pa[e] = lf[e] = rt[e] = -1;
            pv[e] = tl;
            tl = e;
        }
        treeify(hd);
        irregular.insert(idx);
        recode_bin(idx);
    }
    int32_t root_of(int32_t r) const {
        while (pa[r] >= 0) r = pa[r];
        return r;
    }
    // String keys order by spread hash, then String.compareTo
    int dir_for(int32_t x, int32_t p) const {
        if (h[p] > h[x]) return -1;
        if (h[p] < h[x]) return 1;
        return cmp(x, p);
    }
    void treeify(int32_t head) {
        int32_t root = -1;
        for (int32_t x = head, n; x >= 0; x = n) {
            n = nx[x];
            lf[x] = rt[x] = -1;
            if (root < 0) {
                pa[x] = -1;
                set_red(x, false);
                root = x;
                continue;
            }
            for (int32_t p = root;;) {
                const int dir = dir_for(x, p);
                const int32_t xp = p;
                p = dir <= 0 ? lf[p] : rt[p];
                if (p < 0) {
                    pa[x] = xp;
                    if (dir <= 0) lf[xp] = x;
                    else rt[xp] = x;
                    root = balance_insertion(root, x);
                    break;
                }
            }
        }
        move_root_to_front(root);
    }
    int32_t untreeify(int32_t head) {
        for (int32_t q = head; q >= 0; q = nx[q]) {
            fl[q] &= 1;
            pa[q] = lf[q] = rt[q] = pv[q] = -1;
        }
        return head;
    }
    void put_tree_val(int32_t first, int32_t x) {
        const int32_t root = pa[first] >= 0 ? root_of(first) : first;
        fl[x] = 1 | 2;
        for (int32_t p = root;;) {
            const int dir = dir_for(x, p);
            const int32_t xp = p;
            p = dir <= 0 ? lf[p] : rt[p];
            if (p < 0) {
                const int32_t xpn = nx[xp];
                nx[x] = xpn;  // linked right after its tree parent
                if (dir <= 0) lf[xp] = x;
                else rt[xp] = x;
                nx[xp] = x;
                pa[x] = pv[x] = xp;
                if (xpn >= 0) pv[xpn] = x;
                move_root_to_front(balance_insertion(root, x));
                return;
            }
        }
    }
    void move_root_to_front(int32_t root) {
        if (root < 0 || tab.empty()) return;
        const int idx = bin_of(root);
        const int32_t first = tab[idx];
        if (root == first) return;
        tab[idx] = root;
        const int32_t rp = pv[root], rn = nx[root];
        if (rn >= 0) pv[rn] = rp;
        if (rp >= 0) nx[rp] = rn;
        if (first >= 0) pv[first] = root;
        nx[root] = first;
        pv[root] = -1;
    }
    int32_t rotate_left(int32_t root, int32_t p) {
        int32_t r, pp, rl;
        if (p >= 0 && (r = rt[p]) >= 0) {
            rl = rt[p] = lf[r];
            if (rl >= 0) pa[rl] = p;
            pp = pa[r] = pa[p];
            if (pp < 0) {
                root = r;
                set_red(r, false);
            } else if (lf[pp] == p) {
                lf[pp] = r;
            } else {
                rt[pp] = r;
            }
            lf[r] = p;
            pa[p] = r;
        }
        return root;
    }
    int32_t rotate_right(int32_t root, int32_t p) {
        int32_t l, pp, lr;
        if (p >= 0 && (l = lf[p]) >= 0) {
            lr = lf[p] = rt[l];
            if (lr >= 0) pa[lr] = p;
            pp = pa[l] = pa[p];
            if (pp < 0) {
                root = l;
                set_red(l, false);
            } else if (rt[pp] == p) {
                rt[pp] = l;
            } else {
                lf[pp] = l;
            }
            rt[l] = p;
            pa[p] = l;
        }
        return root;
    }
    int32_t balance_insertion(int32_t root, int32_t x) {
        set_red(x, true);
        for (;;) {
            int32_t xp = pa[x], xpp, xppl, xppr;
            if (xp < 0) {
                set_red(x, false);
                return x;
            }
            if (!red(xp) || (xpp = pa[xp]) < 0) return root;
            if (xp == (xppl = lf[xpp])) {
                if ((xppr = rt[xpp]) >= 0 && red(xppr)) {
                    set_red(xppr, false);
                    set_red(xp, false);
                    set_red(xpp, true);
                    x = xpp;
                } else {
                    if (x == rt[xp]) {
                        root = rotate_left(root, x = xp);
                        xp = pa[x];
                        xpp = xp < 0 ? -1 : pa[xp];
                    }
                    if (xp >= 0) {
                        set_red(xp, false);
                        if (xpp >= 0) {
                            set_red(xpp, true);
                            root = rotate_right(root, xpp);
                        }
                    }
                }
            } else {
                if (xppl >= 0 && red(xppl)) {
                    set_red(xppl, false);
                    set_red(xp, false);
                    set_red(xpp, true);
                    x = xpp;
                } else {
                    if (x == lf[xp]) {
                        root = rotate_right(root, x = xp);
                        xp = pa[x];
                        xpp = xp < 0 ? -1 : pa[xp];
                    }
                    if (xp >= 0) {
                        set_red(xp, false);
                        if (xpp >= 0) {
                            set_red(xpp, true);
                            root = rotate_left(root, xpp);
                        }
                    }
                }
            }
        }
    }
    int32_t balance_deletion(int32_t root, int32_t x) {
        for (;;) {
            int32_t xp, xpl, xpr;
            if (x < 0 || x == root) return root;
            if ((xp = pa[x]) < 0) {
                set_red(x, false);
                return x;
            }
            if (red(x)) {
                set_red(x, false);
                return root;
            }
            if ((xpl = lf[xp]) == x) {
                if ((xpr = rt[xp]) >= 0 && red(xpr)) {
                    set_red(xpr, false);
                    set_red(xp, true);
                    root = rotate_left(root, xp);
                    xp = pa[x];
                    xpr = xp < 0 ? -1 : rt[xp];
                }
                if (xpr < 0) {
                    x = xp;
                } else {
                    int32_t sl = lf[xpr], sr = rt[xpr];
                    if ((sr < 0 || !red(sr)) && (sl < 0 || !red(sl))) {
                        set_red(xpr, true);
                        x = xp;
                    } else {
                        if (sr < 0 || !red(sr)) {
                            if (sl >= 0) set_red(sl, false);
                            set_red(xpr, true);
                            root = rotate_right(root, xpr);
                            xp = pa[x];
                            xpr = xp < 0 ? -1 : rt[xp];
                        }
                        if (xpr >= 0) {
                            set_red(xpr, xp >= 0 ? red(xp) : false);
                            if ((sr = rt[xpr]) >= 0) set_red(sr, false);
                        }
                        if (xp >= 0) {
                            set_red(xp, false);
                            root = rotate_left(root, xp);
                        }
                        x = root;
                    }
                }
            } else {
                if (xpl >= 0 && red(xpl)) {
                    set_red(xpl, false);
                    set_red(xp, true);
                    root = rotate_right(root, xp);
                    xp = pa[x];
                    xpl = xp < 0 ? -1 : lf[xp];
                }
                if (xpl < 0) {
                    x = xp;
                } else {
                    int32_t sl = lf[xpl], sr = rt[xpl];
                    if ((sl < 0 || !red(sl)) && (sr < 0 || !red(sr))) {
                        set_red(xpl, true);
                        x = xp;
                    } else {
                        if (sl < 0 || !red(sl)) {
                            if (sr >= 0) set_red(sr, false);
                            set_red(xpl, true);
                            root = rotate_left(root, xpl);
                            xp = pa[x];
                            xpl = xp < 0 ? -1 : lf[xp];
                        }
                        if (xpl >= 0) {
                            set_red(xpl, xp >= 0 ? red(xp) : false);
                            if ((sl = lf[xpl]) >= 0) set_red(sl, false);
                        }
                        if (xp >= 0) {
                            set_red(xp, false);
                            root = rotate_right(root, xp);
                        }
                        x = root;
                    }
                }
            }
        }
    }
    void remove_tree_node(int32_t self, bool movable) {
        const int idx = bin_of(self);
        int32_t first = tab[idx], root = first, rl;
        const int32_t succ = nx[self], pred = pv[self];
        if (pred < 0) tab[idx] = first = succ;
        else nx[pred] = succ;
        if (succ >= 0) pv[succ] = pred;
        if (first < 0) return;
        if (pa[root] >= 0) root = root_of(root);
        if (root < 0 || (movable && (rt[root] < 0 || (rl = lf[root]) < 0 || lf[rl] < 0))) {
            tab[idx] = untreeify(first);  // too small
            return;
        }
        int32_t p = self, pl = lf[self], pr = rt[self], replacement;
        if (pl >= 0 && pr >= 0) {
            int32_t s = pr, sl;
            while ((sl = lf[s]) >= 0) s = sl;  // successor
            const bool c = red(s);
            set_red(s, red(p));
            set_red(p, c);
            const int32_t sr = rt[s];
            const int32_t pp = pa[p];
            if (s == pr) {
                pa[p] = s;
                rt[s] = p;
            } else {
                const int32_t sp = pa[s];
                if ((pa[p] = sp) >= 0) {
                    if (s == lf[sp]) lf[sp] = p;
                    else rt[sp] = p;
                }
                if ((rt[s] = pr) >= 0) pa[pr] = s;
            }
            lf[p] = -1;
            if ((rt[p] = sr) >= 0) pa[sr] = p;
            if ((lf[s] = pl) >= 0) pa[pl] = s;
            if ((pa[s] = pp) < 0) root = s;
            else if (p == lf[pp]) lf[pp] = s;
            else rt[pp] = s;
            replacement = sr >= 0 ? sr : p;
        } else if (pl >= 0) {
            replacement = pl;
        } else if (pr >= 0) {
            replacement = pr;
        } else {
            replacement = p;
        }
        if (replacement != p) {
            const int32_t pp = pa[replacement] = pa[p];
            if (pp < 0) root = replacement;
            else if (p == lf[pp]) lf[pp] = replacement;
            else rt[pp] = replacement;
            lf[p] = rt[p] = pa[p] = -1;
        }
        const int32_t r = red(p) ? root : balance_deletion(root, replacement);
        if (replacement == p) {  // detach
            const int32_t pp = pa[p];
            pa[p] = -1;
            if (pp >= 0) {
                if (p == lf[pp]) lf[pp] = -1;
                else if (p == rt[pp]) rt[pp] = -1;
            }
        }
        if (movable) move_root_to_front(r);
    }
    void split(int32_t b, int index, int bit) {
        int32_t lo_h = -1, lo_t = -1, hi_h = -1, hi_t = -1;
        int lc = 0, hc = 0;
        for (int32_t e = b, n; e >= 0; e = n) {
            n = nx[e];
            nx[e] = -1;
            if ((h[e] & bit) == 0) {
                if ((pv[e] = lo_t) < 0) lo_h = e;
                else nx[lo_t] = e;
                lo_t = e;
                ++lc;
            } else {
                if ((pv[e] = hi_t) < 0) hi_h = e;
                else nx[hi_t] = e;
                hi_t = e;
                ++hc;
            }
        }
        if (lo_h >= 0) {
            if (lc <= kUntreeify) {
                tab[index] = untreeify(lo_h);
            } else {
                tab[index] = lo_h;
                if (hi_h >= 0) treeify(lo_h);
            }
        }
        if (hi_h >= 0) {
            if (hc <= kUntreeify) {
                tab[index + bit] = untreeify(hi_h);
            } else {
                tab[index + bit] = hi_h;
                if (lo_h >= 0) treeify(hi_h);
            }
        }
    }
};

// String.hashCode over UTF-16 code units (int arithmetic)
inline int32_t sh_java_string_hash(const uint16_t* s, int64_t n) {
    uint32_t x = 0;
    for (int64_t i = 0; i < n; i++) x = 31u * x + s[i];
    return (int32_t)x;
}

// The scheduler maps of one app (one per absent pre-state, id = query *
// NF_MAX_PROC + proc) plus the partition keys' toString() they hash.
struct ShSchedModels {
    std::vector<ShJMap> maps;
    std::vector<int> used;                 // scheduler ids in use
    // attr.toString() of each key id (UTF-16, flat); unregistered ids read as
    // their decimal digits
    std::vector<uint16_t> chars;
    std::vector<int64_t> off, len;         // per key: offset into chars, length (-1: unregistered)
    std::vector<int32_t> hash;

    void init(const std::vector<int>& ids, int n_ids) {
        maps.clear();
        maps.resize(n_ids);
        used = ids;
        for (int s : ids) maps[s].cmp = [this](int32_t a, int32_t b) { return compare(a, b); };
    }
    void set_keys(int32_t first, int32_t n, const uint16_t* utf16, const int64_t* offsets) {
        const size_t need = (size_t)first + (size_t)n;
        if (off.size() < need) {
            off.resize(need, 0);
            len.resize(need, -1);
            hash.resize(need, 0);
        }
        for (int32_t i = 0; i < n; i++) {
            const int64_t l = offsets[i + 1] - offsets[i];
            off[first + i] = (int64_t)chars.size();
            len[first + i] = l;
            chars.insert(chars.end(), utf16 + offsets[i], utf16 + offsets[i + 1]);
            hash[first + i] = sh_java_string_hash(utf16 + offsets[i], l);
        }
    }
    void key_string(int32_t k, std::vector<uint16_t>& out) const {
        out.clear();
        if (k < (int32_t)len.size() && len[k] >= 0) {
            out.assign(chars.begin() + off[k], chars.begin() + off[k] + len[k]);
            return;
        }
        char d[16];
        const int n = snprintf(d, sizeof(d), "%d", (int)k);
        for (int i = 0; i < n; i++) out.push_back((uint16_t)d[i]);
    }
    int32_t hash_of(int32_t k) const {
        if (k < (int32_t)len.size() && len[k] >= 0) return hash[k];
        std::vector<uint16_t> s;
        key_string(k, s);
        return sh_java_string_hash(s.data(), (int64_t)s.size());
    }
    // String.compareTo
    int compare(int32_t a, int32_t b) const {
        std::vector<uint16_t> x, y;
        key_string(a, x);
        key_string(b, y);
        const size_t lim = std::min(x.size(), y.size());
        for (size_t i = 0; i < lim; i++)
            if (x[i] != y[i]) return (int)x[i] - (int)y[i];
        return (int)x.size() - (int)y.size();
    }

    // One launch's scheduler history (2 words per record: stamp, key | sched <<
    // 32 | kind << 48) replayed in processing order; a timer launch's removals
    // (returnAllStates) follow all of its getState calls, in iteration order.
    // Returns false when a map outgrew the rank encoding.
    bool apply(const uint64_t* recs, size_t n) {
        std::vector<size_t> ix(n);
        for (size_t i = 0; i < n; i++) ix[i] = i;
        std::stable_sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return recs[2 * a] < recs[2 * b]; });
        std::vector<std::vector<int32_t>> rem(maps.size());
        for (size_t i : ix) {
            const uint64_t w = recs[2 * i + 1];
            const int32_t key = (int32_t)(uint32_t)w;
            const int s = (int)((w >> 32) & 0xFFFF);
            const int kind = (int)(w >> 48);
            if (s >= (int)maps.size()) continue;
            ShJMap& M = maps[s];
            if (kind == 0) {
                M.ensure(key);
                M.set_hash(key, hash_of(key));
                M.compute_if_absent(key);
            } else if (kind == 1) {
                M.touch();
            } else {
                rem[s].push_back(key);
            }
        }
        for (size_t s = 0; s < maps.size(); s++) {
            if (rem[s].empty()) continue;
            maps[s].sort_iteration(rem[s]);
            for (int32_t k : rem[s]) maps[s].remove(k, false);
        }
        for (int s : used)
            if (!maps[s].rank_fits()) return false;
        return true;
    }
};
