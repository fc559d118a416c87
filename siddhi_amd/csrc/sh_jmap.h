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
#include <stdlib.h>

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
    // one record per key (a key's fields share a cache line: the replay's accesses
    // are random over up to 10M keys)
    struct Node {
        uint64_t code;             // position code (rank = bucket << 38 | code)
        int32_t h;                 // spread hash (registered once per key)
        int32_t nx, pv, pa, lf, rt;
        uint8_t fl;                // 1 present, 2 tree node, 4 red, 8 hash set (kept across removal)
    };
    std::vector<Node> nd;
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
        if (k < (int32_t)nd.size()) return;
        const size_t n = std::max<size_t>((size_t)k + 1, nd.size() * 2);
        nd.resize(n, Node{0, 0, -1, -1, -1, -1, -1, 0});
    }
    static int32_t spread(int32_t x) { return x ^ (int32_t)((uint32_t)x >> 16); }
    void set_hash(int32_t k, int32_t string_hash) {
        ensure(k);
        nd[k].h = spread(string_hash);
        nd[k].fl |= 8;
    }
    bool hashed(int32_t k) const { return k < (int32_t)nd.size() && (nd[k].fl & 8); }
    // the replay's look-ahead: a key's node, then (hash set) its bin head
    void prefetch_node(int32_t k) const {
        if (k >= 0 && k < (int32_t)nd.size()) __builtin_prefetch(&nd[k], 1);
    }
    void prefetch_bin(int32_t k) const {
        if (k >= 0 && k < (int32_t)nd.size() && (nd[k].fl & 8) && !tab.empty())
            __builtin_prefetch(&tab[(size_t)((cap() - 1) & nd[k].h)], 1);
    }
    bool present(int32_t k) const { return k < (int32_t)nd.size() && (nd[k].fl & 1); }
    bool is_tree(int32_t k) const { return (nd[k].fl & 2) != 0; }
    bool red(int32_t k) const { return k >= 0 && (nd[k].fl & 4) != 0; }
    void set_red(int32_t k, bool r) {
        if (r) nd[k].fl |= 4;
        else nd[k].fl &= (uint8_t)~4;
    }
    int cap() const { return (int)tab.size(); }
    int bin_of(int32_t k) const { return (cap() - 1) & nd[k].h; }
    uint64_t rank(int32_t k) const { return ((uint64_t)(uint32_t)bin_of(k) << 38) | nd[k].code; }
    bool rank_fits() const { return cap() <= (1 << kRankBucketBits); }

    // list positions of an irregular bin become its codes
    void recode_bin(int b) {
        uint64_t pos = 0;
        for (int32_t e = tab[b]; e >= 0; e = nd[e].nx) {
            nd[e].code = pos++;
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
            for (int32_t e = first; e >= 0; e = nd[e].nx) ++bin_count;
        nd[k].fl = (uint8_t)((nd[k].fl & 8) | 1);
        nd[k].pa = nd[k].lf = nd[k].rt = nd[k].pv = -1;
        if (tree_bin) {
            put_tree_val(first, k);
            irregular.insert(i);
            recode_bin(i);
        } else {
            nd[k].nx = first;  // newNode(hash, key, value, first): the new head
            tab[i] = k;
            nd[k].code = kMaxCode - (ord++ & kMaxCode);
            dirty.push_back(k);
            if (bin_count >= kTreeify - 1) treeify_bin(nd[k].h);
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
            tab[idx] = nd[k].nx;
        } else {
            int32_t p = tab[idx];
            while (nd[p].nx != k) p = nd[p].nx;
            nd[p].nx = nd[k].nx;
        }
        nd[k].fl &= 8;
        nd[k].nx = nd[k].pv = nd[k].pa = nd[k].lf = nd[k].rt = -1;
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
                for (int32_t e = tab[bin_of(k)]; e >= 0 && e != k; e = nd[e].nx) ++pos;
            } else if (present(k)) {
                pos = nd[k].code;
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
            if (nd[e].nx < 0) {
                tab[nd[e].h & (new_cap - 1)] = e;
                if (irr) mark_irregular(nd[e].h & (new_cap - 1));
            } else if (is_tree(e)) {
                split(e, j, old_cap);
                mark_irregular(j);
                mark_irregular(j + old_cap);
            } else {
                int32_t lo_h = -1, lo_t = -1, hi_h = -1, hi_t = -1;
                for (int32_t x = e; x >= 0;) {
                    const int32_t n = nd[x].nx;
                    if ((nd[x].h & old_cap) == 0) {
                        if (lo_t < 0) lo_h = x;
                        else nd[lo_t].nx = x;
                        lo_t = x;
                    } else {
                        if (hi_t < 0) hi_h = x;
                        else nd[hi_t].nx = x;
                        hi_t = x;
                    }
                    x = n;
                }
                if (lo_t >= 0) {
                    nd[lo_t].nx = -1;
                    tab[j] = lo_h;
                }
                if (hi_t >= 0) {
                    nd[hi_t].nx = -1;
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
        for (int32_t e = hd; e >= 0; e = nd[e].nx) {  // replacementTreeNode: same list order
            nd[e].fl = (uint8_t)((nd[e].fl & 9) | 2);
            nd[e].pa = nd[e].lf = nd[e].rt = -1;
            nd[e].pv = tl;
            tl = e;
        }
        treeify(hd);
        irregular.insert(idx);
        recode_bin(idx);
    }
    int32_t root_of(int32_t r) const {
        while (nd[r].pa >= 0) r = nd[r].pa;
        return r;
    }
    // String keys order by spread hash, then String.compareTo
    int dir_for(int32_t x, int32_t p) const {
        if (nd[p].h > nd[x].h) return -1;
        if (nd[p].h < nd[x].h) return 1;
        return cmp(x, p);
    }
    void treeify(int32_t head) {
        int32_t root = -1;
        for (int32_t x = head, n; x >= 0; x = n) {
            n = nd[x].nx;
            nd[x].lf = nd[x].rt = -1;
            if (root < 0) {
                nd[x].pa = -1;
                set_red(x, false);
                root = x;
                continue;
            }
            for (int32_t p = root;;) {
                const int dir = dir_for(x, p);
                const int32_t xp = p;
                p = dir <= 0 ? nd[p].lf : nd[p].rt;
                if (p < 0) {
                    nd[x].pa = xp;
                    if (dir <= 0) nd[xp].lf = x;
                    else nd[xp].rt = x;
                    root = balance_insertion(root, x);
                    break;
                }
            }
        }
        move_root_to_front(root);
    }
    int32_t untreeify(int32_t head) {
        for (int32_t q = head; q >= 0; q = nd[q].nx) {
            nd[q].fl &= 9;
            nd[q].pa = nd[q].lf = nd[q].rt = nd[q].pv = -1;
        }
        return head;
    }
    void put_tree_val(int32_t first, int32_t x) {
        const int32_t root = nd[first].pa >= 0 ? root_of(first) : first;
        nd[x].fl = (uint8_t)((nd[x].fl & 8) | 1 | 2);
        for (int32_t p = root;;) {
            const int dir = dir_for(x, p);
            const int32_t xp = p;
            p = dir <= 0 ? nd[p].lf : nd[p].rt;
            if (p < 0) {
                const int32_t xpn = nd[xp].nx;
                nd[x].nx = xpn;  // linked right after its tree parent
                if (dir <= 0) nd[xp].lf = x;
                else nd[xp].rt = x;
                nd[xp].nx = x;
                nd[x].pa = nd[x].pv = xp;
                if (xpn >= 0) nd[xpn].pv = x;
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
        const int32_t rp = nd[root].pv, rn = nd[root].nx;
        if (rn >= 0) nd[rn].pv = rp;
        if (rp >= 0) nd[rp].nx = rn;
        if (first >= 0) nd[first].pv = root;
        nd[root].nx = first;
        nd[root].pv = -1;
    }
    int32_t rotate_left(int32_t root, int32_t p) {
        int32_t r, pp, rl;
        if (p >= 0 && (r = nd[p].rt) >= 0) {
            rl = nd[p].rt = nd[r].lf;
            if (rl >= 0) nd[rl].pa = p;
            pp = nd[r].pa = nd[p].pa;
            if (pp < 0) {
                root = r;
                set_red(r, false);
            } else if (nd[pp].lf == p) {
                nd[pp].lf = r;
            } else {
                nd[pp].rt = r;
            }
            nd[r].lf = p;
            nd[p].pa = r;
        }
        return root;
    }
    int32_t rotate_right(int32_t root, int32_t p) {
        int32_t l, pp, lr;
        if (p >= 0 && (l = nd[p].lf) >= 0) {
            lr = nd[p].lf = nd[l].rt;
            if (lr >= 0) nd[lr].pa = p;
            pp = nd[l].pa = nd[p].pa;
            if (pp < 0) {
                root = l;
                set_red(l, false);
            } else if (nd[pp].rt == p) {
                nd[pp].rt = l;
            } else {
                nd[pp].lf = l;
            }
            nd[l].rt = p;
            nd[p].pa = l;
        }
        return root;
    }
    int32_t balance_insertion(int32_t root, int32_t x) {
        set_red(x, true);
        for (;;) {
            int32_t xp = nd[x].pa, xpp, xppl, xppr;
            if (xp < 0) {
                set_red(x, false);
                return x;
            }
            if (!red(xp) || (xpp = nd[xp].pa) < 0) return root;
            if (xp == (xppl = nd[xpp].lf)) {
                if ((xppr = nd[xpp].rt) >= 0 && red(xppr)) {
                    set_red(xppr, false);
                    set_red(xp, false);
                    set_red(xpp, true);
                    x = xpp;
                } else {
                    if (x == nd[xp].rt) {
                        root = rotate_left(root, x = xp);
                        xp = nd[x].pa;
                        xpp = xp < 0 ? -1 : nd[xp].pa;
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
                    if (x == nd[xp].lf) {
                        root = rotate_right(root, x = xp);
                        xp = nd[x].pa;
                        xpp = xp < 0 ? -1 : nd[xp].pa;
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
            if ((xp = nd[x].pa) < 0) {
                set_red(x, false);
                return x;
            }
            if (red(x)) {
                set_red(x, false);
                return root;
            }
            if ((xpl = nd[xp].lf) == x) {
                if ((xpr = nd[xp].rt) >= 0 && red(xpr)) {
                    set_red(xpr, false);
                    set_red(xp, true);
                    root = rotate_left(root, xp);
                    xp = nd[x].pa;
                    xpr = xp < 0 ? -1 : nd[xp].rt;
                }
                if (xpr < 0) {
                    x = xp;
                } else {
                    int32_t sl = nd[xpr].lf, sr = nd[xpr].rt;
                    if ((sr < 0 || !red(sr)) && (sl < 0 || !red(sl))) {
                        set_red(xpr, true);
                        x = xp;
                    } else {
                        if (sr < 0 || !red(sr)) {
                            if (sl >= 0) set_red(sl, false);
                            set_red(xpr, true);
                            root = rotate_right(root, xpr);
                            xp = nd[x].pa;
                            xpr = xp < 0 ? -1 : nd[xp].rt;
                        }
                        if (xpr >= 0) {
                            set_red(xpr, xp >= 0 ? red(xp) : false);
                            if ((sr = nd[xpr].rt) >= 0) set_red(sr, false);
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
                    xp = nd[x].pa;
                    xpl = xp < 0 ? -1 : nd[xp].lf;
                }
                if (xpl < 0) {
                    x = xp;
                } else {
                    int32_t sl = nd[xpl].lf, sr = nd[xpl].rt;
                    if ((sl < 0 || !red(sl)) && (sr < 0 || !red(sr))) {
                        set_red(xpl, true);
                        x = xp;
                    } else {
                        if (sl < 0 || !red(sl)) {
                            if (sr >= 0) set_red(sr, false);
                            set_red(xpl, true);
                            root = rotate_left(root, xpl);
                            xp = nd[x].pa;
                            xpl = xp < 0 ? -1 : nd[xp].lf;
                        }
                        if (xpl >= 0) {
                            set_red(xpl, xp >= 0 ? red(xp) : false);
                            if ((sl = nd[xpl].lf) >= 0) set_red(sl, false);
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
        const int32_t succ = nd[self].nx, pred = nd[self].pv;
        if (pred < 0) tab[idx] = first = succ;
        else nd[pred].nx = succ;
        if (succ >= 0) nd[succ].pv = pred;
        if (first < 0) return;
        if (nd[root].pa >= 0) root = root_of(root);
        if (root < 0 || (movable && (nd[root].rt < 0 || (rl = nd[root].lf) < 0 || nd[rl].lf < 0))) {
            tab[idx] = untreeify(first);  // too small
            return;
        }
        int32_t p = self, pl = nd[self].lf, pr = nd[self].rt, replacement;
        if (pl >= 0 && pr >= 0) {
            int32_t s = pr, sl;
            while ((sl = nd[s].lf) >= 0) s = sl;  // successor
            const bool c = red(s);
            set_red(s, red(p));
            set_red(p, c);
            const int32_t sr = nd[s].rt;
            const int32_t pp = nd[p].pa;
            if (s == pr) {
                nd[p].pa = s;
                nd[s].rt = p;
            } else {
                const int32_t sp = nd[s].pa;
                if ((nd[p].pa = sp) >= 0) {
                    if (s == nd[sp].lf) nd[sp].lf = p;
                    else nd[sp].rt = p;
                }
                if ((nd[s].rt = pr) >= 0) nd[pr].pa = s;
            }
            nd[p].lf = -1;
            if ((nd[p].rt = sr) >= 0) nd[sr].pa = p;
            if ((nd[s].lf = pl) >= 0) nd[pl].pa = s;
            if ((nd[s].pa = pp) < 0) root = s;
            else if (p == nd[pp].lf) nd[pp].lf = s;
            else nd[pp].rt = s;
            replacement = sr >= 0 ? sr : p;
        } else if (pl >= 0) {
            replacement = pl;
        } else if (pr >= 0) {
            replacement = pr;
        } else {
            replacement = p;
        }
        if (replacement != p) {
            const int32_t pp = nd[replacement].pa = nd[p].pa;
            if (pp < 0) root = replacement;
            else if (p == nd[pp].lf) nd[pp].lf = replacement;
            else nd[pp].rt = replacement;
            nd[p].lf = nd[p].rt = nd[p].pa = -1;
        }
        const int32_t r = red(p) ? root : balance_deletion(root, replacement);
        if (replacement == p) {  // detach
            const int32_t pp = nd[p].pa;
            nd[p].pa = -1;
            if (pp >= 0) {
                if (p == nd[pp].lf) nd[pp].lf = -1;
                else if (p == nd[pp].rt) nd[pp].rt = -1;
            }
        }
        if (movable) move_root_to_front(r);
    }
    void split(int32_t b, int index, int bit) {
        int32_t lo_h = -1, lo_t = -1, hi_h = -1, hi_t = -1;
        int lc = 0, hc = 0;
        for (int32_t e = b, n; e >= 0; e = n) {
            n = nd[e].nx;
            nd[e].nx = -1;
            if ((nd[e].h & bit) == 0) {
                if ((nd[e].pv = lo_t) < 0) lo_h = e;
                else nd[lo_t].nx = e;
                lo_t = e;
                ++lc;
            } else {
                if ((nd[e].pv = hi_t) < 0) hi_h = e;
                else nd[hi_t].nx = e;
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
    // false: some id in [first, first + n) already sits in a map under the hash of
    // another string (it was used before its string was registered; its bin -- and
    // so the due-timer tie order -- would stay that of the old string)
    bool keys_settable(int32_t first, int32_t n, const uint16_t* utf16, const int64_t* offsets) const {
        for (int32_t i = 0; i < n; i++) {
            const int32_t k = first + i;
            bool used_k = false;
            for (const ShJMap& M : maps) used_k = used_k || M.hashed(k);
            if (!used_k) continue;
            const int32_t nh = sh_java_string_hash(utf16 + offsets[i], offsets[i + 1] - offsets[i]);
            if (nh != hash_of(k)) return false;
        }
        return true;
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
        // the records touch random keys of up to 10M: look ahead in the (fixed)
        // replay order -- the node kPfNode records ahead, its bin head (or its
        // string hash, first sight of the key) kPfBin ahead
        const size_t kPfNode = 16, kPfBin = 8;
        auto pf = [&](size_t j, bool node) {
            const uint64_t w = recs[2 * ix[j] + 1];
            const int s = (int)((w >> 32) & 0xFFFF);
            if ((w >> 48) != 0 || s >= (int)maps.size()) return;
            const int32_t key = (int32_t)(uint32_t)w;
            if (node) {
                maps[s].prefetch_node(key);
            } else if (maps[s].hashed(key)) {
                maps[s].prefetch_bin(key);
            } else if (key >= 0 && key < (int32_t)hash.size()) {
                __builtin_prefetch(&hash[key]);
                __builtin_prefetch(&len[key]);
            }
        };
        static const bool pf_on = !(getenv("SH_HIST_PF") && getenv("SH_HIST_PF")[0] == '0');
        for (size_t j = 0; j < n; j++) {
            if (pf_on && j + kPfNode < n) pf(j + kPfNode, true);
            if (pf_on && j + kPfBin < n) pf(j + kPfBin, false);
            const size_t i = ix[j];
            const uint64_t w = recs[2 * i + 1];
            const int32_t key = (int32_t)(uint32_t)w;
            const int s = (int)((w >> 32) & 0xFFFF);
            const int kind = (int)(w >> 48);
            if (s >= (int)maps.size()) continue;
            ShJMap& M = maps[s];
            if (kind == 0) {
                M.ensure(key);
                if (!M.hashed(key)) M.set_hash(key, hash_of(key));
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
