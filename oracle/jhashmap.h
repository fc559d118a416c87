// jhashmap.h — CPU ORACLE (test infrastructure): a restatement of
// java.util.HashMap (OpenJDK 8u, java/util/HashMap.java) for String keys, kept
// only for its ITERATION ORDER. siddhi-core's playback Scheduler walks
// PartitionStateHolder.states, a HashMap<String, Map<String, State>>
// (util/snapshot/state/PartitionStateHolder.java:36), in that order and keeps one
// SchedulerState per due time (util/Scheduler.java:75-87, compareTo()==0 at
// :364-366), so which partition key fires depends on bucket order.
//
// The JDK is a third-party dependency absent from /root/reference (no JDK in
// this image); the restated operations are the published OpenJDK 8 code paths
// the reference exercises:
//   computeIfAbsent   PartitionStateHolder.getState (:46): lazy resize when
//                     size > threshold on ANY call, new node at the HEAD of its
//                     bin, treeifyBin when the bin already held >= 7 nodes
//                     (resize instead while the table is < 64)
//   remove(key)       PartitionStateHolder.removeState (:76): removeNode(movable)
//   iterator.remove   PartitionStateHolder.returnAllStates (:159):
//                     removeNode(..., movable = false)
//   resize / split    lo/hi split preserving order; tree bins re-treeified, or
//                     untreeified when a half has <= 6 nodes
//   TreeNode          treeify, putTreeVal (new node linked after its tree
//                     parent), moveRootToFront, balanceInsertion,
//                     removeTreeNode, balanceDeletion, rotations; String keys
//                     order by hash then String.compareTo (UTF-16 code units)
// Keys are dense key ids; their String (attr.toString()) is supplied by the caller.
#pragma once
#include <stdint.h>

#include <functional>
#include <unordered_map>
#include <vector>

namespace ref {

struct JNode {
    int32_t hash = 0;  // spread hash: h ^ (h >>> 16)
    int64_t key = 0;
    JNode* next = nullptr;
    // TreeNode (LinkedHashMap.Entry before/after are unused by HashMap)
    bool tree = false;
    JNode* parent = nullptr;
    JNode* left = nullptr;
    JNode* right = nullptr;
    JNode* prev = nullptr;
    bool red = false;
};

class JHashMap {
   public:
    // String.compareTo(key a, key b) and String.hashCode(key)
    std::function<int(int64_t, int64_t)> compare;
    std::function<int32_t(int64_t)> string_hash;

    ~JHashMap() {
        for (auto& kv : where_) delete kv.second;
    }
    int size() const { return size_; }
    int capacity() const { return (int)table_.size(); }
    bool contains(int64_t k) const { return where_.count(k) != 0; }

    // HashMap.computeIfAbsent(key, f) with a non-null f: true when a node was added
    bool computeIfAbsent(int64_t key) {
        const int32_t hash = spread(string_hash(key));
        if (size_ > threshold_ || table_.empty()) resize();
        int n = (int)table_.size();
        int i = (n - 1) & hash;
        JNode* first = table_[i];
        int binCount = 0;
        JNode* t = nullptr;
        if (first) {
            if (first->tree) {
                t = first;
                if (where_.count(key)) return false;  // getTreeNode found it
            } else {
                for (JNode* e = first; e; e = e->next) {
                    if (e->key == key) return false;
                    ++binCount;
                }
            }
        }
        JNode* x = new JNode();
        x->hash = hash;
        x->key = key;
        where_[key] = x;
        if (t) {
            putTreeVal(t, x);
        } else {
            x->next = first;  // newNode(hash, key, v, first)
            table_[i] = x;
            if (binCount >= kTreeifyThreshold - 1) treeifyBin(hash);
        }
        ++size_;
        return true;
    }

    // HashMap.removeNode(hash(key), key, null, false, movable)
    bool remove(int64_t key, bool movable) {
        auto it = where_.find(key);
        if (it == where_.end() || table_.empty()) return false;
        JNode* node = it->second;
        const int n = (int)table_.size();
        const int index = (n - 1) & node->hash;
        JNode* p = table_[index];
        if (node->tree) {
            removeTreeNode(node, movable);
        } else if (node == p) {
            table_[index] = node->next;
        } else {
            while (p->next != node) p = p->next;
            p->next = node->next;
        }
        where_.erase(it);
        delete node;
        --size_;
        return true;
    }

    // keys in iteration order (HashIterator: bins ascending, `next` chains)
    template <class F>
    void forEach(F f) const {
        for (JNode* b : table_)
            for (JNode* e = b; e; e = e->next) f(e->key);
    }
    std::vector<int64_t> keys() const {
        std::vector<int64_t> out;
        out.reserve(size_);
        forEach([&](int64_t k) { out.push_back(k); });
        return out;
    }

   private:
    static const int kTreeifyThreshold = 8;
    static const int kUntreeifyThreshold = 6;
    static const int kMinTreeifyCapacity = 64;
    static const int kMaxCapacity = 1 << 30;
    std::vector<JNode*> table_;
    int size_ = 0;
    int threshold_ = 0;
    std::unordered_map<int64_t, JNode*> where_;

    static int32_t spread(int32_t h) { return h ^ (int32_t)((uint32_t)h >> 16); }

    // String keys: comparableClassFor(k) == String.class, so ties in hash order
    // by compareTo (distinct keys never compare equal; tieBreakOrder unused)
    int dirFor(const JNode* x, const JNode* p) const {
        if (p->hash > x->hash) return -1;
        if (p->hash < x->hash) return 1;
        return compare(x->key, p->key);
    }

    void resize() {
        const int oldCap = (int)table_.size();
        const int oldThr = threshold_;
        int newCap = 0, newThr = 0;
        if (oldCap > 0) {
            if (oldCap >= kMaxCapacity) {
                threshold_ = 0x7FFFFFFF;
                return;
            }
            newCap = oldCap << 1;
            if (newCap < kMaxCapacity && oldCap >= 16) newThr = oldThr << 1;
        } else if (oldThr > 0) {
            newCap = oldThr;
        } else {
            newCap = 16;
            newThr = 12;
        }
        if (newThr == 0) {
            const float ft = (float)newCap * 0.75f;
            newThr = (newCap < kMaxCapacity && ft < (float)kMaxCapacity) ? (int)ft : 0x7FFFFFFF;
        }
        threshold_ = newThr;
        std::vector<JNode*> oldTab;
        oldTab.swap(table_);
        table_.assign(newCap, nullptr);
        for (int j = 0; j < oldCap; ++j) {
            JNode* e = oldTab[j];
            if (!e) continue;
            if (!e->next) {
                table_[e->hash & (newCap - 1)] = e;
            } else if (e->tree) {
                split(e, j, oldCap);
            } else {
                JNode *loHead = nullptr, *loTail = nullptr, *hiHead = nullptr, *hiTail = nullptr;
                for (JNode* x = e; x;) {
                    JNode* nx = x->next;
                    if ((x->hash & oldCap) == 0) {
                        if (!loTail) loHead = x;
                        else loTail->next = x;
                        loTail = x;
                    } else {
                        if (!hiTail) hiHead = x;
                        else hiTail->next = x;
                        hiTail = x;
                    }
                    x = nx;
                }
                if (loTail) {
                    loTail->next = nullptr;
                    table_[j] = loHead;
                }
                if (hiTail) {
                    hiTail->next = nullptr;
                    table_[j + oldCap] = hiHead;
                }
            }
        }
    }

    void treeifyBin(int32_t hash) {
        const int n = (int)table_.size();
        if (n < kMinTreeifyCapacity) {
            resize();
            return;
        }
        const int index = (n - 1) & hash;
        JNode* e = table_[index];
        if (!e) return;
        JNode *hd = nullptr, *tl = nullptr;
        for (; e; e = e->next) {  // replacementTreeNode keeps the list order
            e->tree = true;
            e->parent = e->left = e->right = nullptr;
            e->red = false;
            e->prev = tl;
            if (!tl) hd = e;
            tl = e;
        }
        table_[index] = hd;
        treeify(hd);
    }

    static JNode* rootOf(JNode* r) {
        while (r->parent) r = r->parent;
        return r;
    }

    void treeify(JNode* head) {
        JNode* root = nullptr;
        for (JNode *x = head, *nx; x; x = nx) {
            nx = x->next;
            x->left = x->right = nullptr;
            if (!root) {
                x->parent = nullptr;
                x->red = false;
                root = x;
            } else {
                for (JNode* p = root;;) {
                    const int dir = dirFor(x, p);
                    JNode* xp = p;
                    if ((p = (dir <= 0) ? p->left : p->right) == nullptr) {
                        x->parent = xp;
                        if (dir <= 0) xp->left = x;
                        else xp->right = x;
                        root = balanceInsertion(root, x);
                        break;
                    }
                }
            }
        }
        moveRootToFront(root);
    }

    JNode* untreeify(JNode* head) {
        for (JNode* q = head; q; q = q->next) {  // replacementNode: same order, plain nodes
            q->tree = false;
            q->parent = q->left = q->right = q->prev = nullptr;
            q->red = false;
        }
        return head;
    }

    void putTreeVal(JNode* binFirst, JNode* x) {
        JNode* root = binFirst->parent ? rootOf(binFirst) : binFirst;
        x->tree = true;
        for (JNode* p = root;;) {
            const int dir = dirFor(x, p);
            JNode* xp = p;
            if ((p = (dir <= 0) ? p->left : p->right) == nullptr) {
                JNode* xpn = xp->next;  // newTreeNode(h, k, v, xpn)
                x->next = xpn;
                if (dir <= 0) xp->left = x;
                else xp->right = x;
                xp->next = x;
                x->parent = x->prev = xp;
                if (xpn) xpn->prev = x;
                moveRootToFront(balanceInsertion(root, x));
                return;
            }
        }
    }

    void moveRootToFront(JNode* root) {
        if (!root || table_.empty()) return;
        const int index = ((int)table_.size() - 1) & root->hash;
        JNode* first = table_[index];
        if (root != first) {
            table_[index] = root;
            JNode* rp = root->prev;
            JNode* rn = root->next;
            if (rn) rn->prev = rp;
            if (rp) rp->next = rn;
            if (first) first->prev = root;
            root->next = first;
            root->prev = nullptr;
        }
    }

    static JNode* rotateLeft(JNode* root, JNode* p) {
        JNode *r, *pp, *rl;
        if (p && (r = p->right)) {
            if ((rl = p->right = r->left)) rl->parent = p;
            if (!(pp = r->parent = p->parent)) {
                root = r;
                r->red = false;
            } else if (pp->left == p) {
                pp->left = r;
            } else {
                pp->right = r;
            }
            r->left = p;
            p->parent = r;
        }
        return root;
    }

    static JNode* rotateRight(JNode* root, JNode* p) {
        JNode *l, *pp, *lr;
        if (p && (l = p->left)) {
            if ((lr = p->left = l->right)) lr->parent = p;
            if (!(pp = l->parent = p->parent)) {
                root = l;
                l->red = false;
            } else if (pp->right == p) {
                pp->right = l;
            } else {
                pp->left = l;
            }
            l->right = p;
            p->parent = l;
        }
        return root;
    }

    static JNode* balanceInsertion(JNode* root, JNode* x) {
        x->red = true;
        for (JNode *xp, *xpp, *xppl, *xppr;;) {
            if (!(xp = x->parent)) {
                x->red = false;
                return x;
            } else if (!xp->red || !(xpp = xp->parent)) {
                return root;
            }
            if (xp == (xppl = xpp->left)) {
                if ((xppr = xpp->right) && xppr->red) {
                    xppr->red = false;
                    xp->red = false;
                    xpp->red = true;
                    x = xpp;
                } else {
                    if (x == xp->right) {
                        root = rotateLeft(root, x = xp);
                        xpp = (xp = x->parent) == nullptr ? nullptr : xp->parent;
                    }
                    if (xp) {
                        xp->red = false;
                        if (xpp) {
                            xpp->red = true;
                            root = rotateRight(root, xpp);
                        }
                    }
                }
            } else {
                if (xppl && xppl->red) {
                    xppl->red = false;
                    xp->red = false;
                    xpp->red = true;
                    x = xpp;
                } else {
                    if (x == xp->left) {
                        root = rotateRight(root, x = xp);
                        xpp = (xp = x->parent) == nullptr ? nullptr : xp->parent;
                    }
                    if (xp) {
                        xp->red = false;
                        if (xpp) {
                            xpp->red = true;
                            root = rotateLeft(root, xpp);
                        }
                    }
                }
            }
        }
    }

    static JNode* balanceDeletion(JNode* root, JNode* x) {
        for (JNode *xp, *xpl, *xpr;;) {
            if (!x || x == root) return root;
            if (!(xp = x->parent)) {
                x->red = false;
                return x;
            } else if (x->red) {
                x->red = false;
                return root;
            } else if ((xpl = xp->left) == x) {
                if ((xpr = xp->right) && xpr->red) {
                    xpr->red = false;
                    xp->red = true;
                    root = rotateLeft(root, xp);
                    xpr = (xp = x->parent) == nullptr ? nullptr : xp->right;
                }
                if (!xpr) {
                    x = xp;
                } else {
                    JNode *sl = xpr->left, *sr = xpr->right;
                    if ((!sr || !sr->red) && (!sl || !sl->red)) {
                        xpr->red = true;
                        x = xp;
                    } else {
                        if (!sr || !sr->red) {
                            if (sl) sl->red = false;
                            xpr->red = true;
                            root = rotateRight(root, xpr);
                            xpr = (xp = x->parent) == nullptr ? nullptr : xp->right;
                        }
                        if (xpr) {
                            xpr->red = xp ? xp->red : false;
                            if ((sr = xpr->right)) sr->red = false;
                        }
                        if (xp) {
                            xp->red = false;
                            root = rotateLeft(root, xp);
                        }
                        x = root;
                    }
                }
            } else {  // symmetric
                if (xpl && xpl->red) {
                    xpl->red = false;
                    xp->red = true;
                    root = rotateRight(root, xp);
                    xpl = (xp = x->parent) == nullptr ? nullptr : xp->left;
                }
                if (!xpl) {
                    x = xp;
                } else {
                    JNode *sl = xpl->left, *sr = xpl->right;
                    if ((!sl || !sl->red) && (!sr || !sr->red)) {
                        xpl->red = true;
                        x = xp;
                    } else {
                        if (!sl || !sl->red) {
                            if (sr) sr->red = false;
                            xpl->red = true;
                            root = rotateLeft(root, xpl);
                            xpl = (xp = x->parent) == nullptr ? nullptr : xp->left;
                        }
                        if (xpl) {
                            xpl->red = xp ? xp->red : false;
                            if ((sl = xpl->left)) sl->red = false;
                        }
                        if (xp) {
                            xp->red = false;
                            root = rotateRight(root, xp);
                        }
                        x = root;
                    }
                }
            }
        }
    }

    // TreeNode.removeTreeNode (the node is unlinked from `next`/`prev` first; a
    // too-small tree is untreeified only when `movable`)
    void removeTreeNode(JNode* self, bool movable) {
        const int n = (int)table_.size();
        const int index = (n - 1) & self->hash;
        JNode* first = table_[index];
        JNode* root = first;
        JNode *succ = self->next, *pred = self->prev, *rl;
        if (!pred) table_[index] = first = succ;
        else pred->next = succ;
        if (succ) succ->prev = pred;
        if (!first) return;
        if (root->parent) root = rootOf(root);
        if (!root || (movable && (!root->right || !(rl = root->left) || !rl->left))) {
            table_[index] = untreeify(first);  // too small
            return;
        }
        JNode *p = self, *pl = self->left, *pr = self->right, *replacement;
        if (pl && pr) {
            JNode *s = pr, *sl;
            while ((sl = s->left)) s = sl;  // successor
            const bool c = s->red;
            s->red = p->red;
            p->red = c;
            JNode* sr = s->right;
            JNode* pp = p->parent;
            if (s == pr) {
                p->parent = s;
                s->right = p;
            } else {
                JNode* sp = s->parent;
                if ((p->parent = sp)) {
                    if (s == sp->left) sp->left = p;
                    else sp->right = p;
                }
                if ((s->right = pr)) pr->parent = s;
            }
            p->left = nullptr;
            if ((p->right = sr)) sr->parent = p;
            if ((s->left = pl)) pl->parent = s;
            if (!(s->parent = pp)) root = s;
            else if (p == pp->left) pp->left = s;
            else pp->right = s;
            replacement = sr ? sr : p;
        } else if (pl) {
            replacement = pl;
        } else if (pr) {
            replacement = pr;
        } else {
            replacement = p;
        }
        if (replacement != p) {
            JNode* pp = replacement->parent = p->parent;
            if (!pp) root = replacement;
            else if (p == pp->left) pp->left = replacement;
            else pp->right = replacement;
            p->left = p->right = p->parent = nullptr;
        }
        JNode* r = p->red ? root : balanceDeletion(root, replacement);
        if (replacement == p) {  // detach
            JNode* pp = p->parent;
            p->parent = nullptr;
            if (pp) {
                if (p == pp->left) pp->left = nullptr;
                else if (p == pp->right) pp->right = nullptr;
            }
        }
        if (movable) moveRootToFront(r);
    }

    // TreeNode.split during resize
    void split(JNode* b, int index, int bit) {
        JNode *loHead = nullptr, *loTail = nullptr, *hiHead = nullptr, *hiTail = nullptr;
        int lc = 0, hc = 0;
        for (JNode *e = b, *nx; e; e = nx) {
            nx = e->next;
            e->next = nullptr;
            if ((e->hash & bit) == 0) {
                if (!(e->prev = loTail)) loHead = e;
                else loTail->next = e;
                loTail = e;
                ++lc;
            } else {
                if (!(e->prev = hiTail)) hiHead = e;
                else hiTail->next = e;
                hiTail = e;
                ++hc;
            }
        }
        if (loHead) {
            if (lc <= kUntreeifyThreshold) {
                table_[index] = untreeify(loHead);
            } else {
                table_[index] = loHead;
                if (hiHead) treeify(loHead);
            }
        }
        if (hiHead) {
            if (hc <= kUntreeifyThreshold) {
                table_[index + bit] = untreeify(hiHead);
            } else {
                table_[index + bit] = hiHead;
                if (loHead) treeify(hiHead);
            }
        }
    }
};

// String.hashCode over UTF-16 code units: s[0]*31^(n-1) + ... + s[n-1] (int arithmetic)
inline int32_t java_string_hash(const uint16_t* s, int64_t n) {
    uint32_t h = 0;
    for (int64_t i = 0; i < n; i++) h = 31u * h + s[i];
    return (int32_t)h;
}

// String.compareTo: first differing UTF-16 code unit, else length difference
inline int java_string_compare(const uint16_t* a, int64_t na, const uint16_t* b, int64_t nb) {
    const int64_t lim = na < nb ? na : nb;
    for (int64_t i = 0; i < lim; i++)
        if (a[i] != b[i]) return (int)a[i] - (int)b[i];
    return (int)(na - nb);
}

}  // namespace ref
