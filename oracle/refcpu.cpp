// refcpu.cpp — CPU ORACLE: a line-by-line C++ restatement of siddhi-core's
// pattern/sequence (NFA) engine. TEST INFRASTRUCTURE ONLY: loaded by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
// The product path (libsiddhi_hip.so) never links or calls this.
//
// Java object semantics are modelled explicitly: StateEvent / StreamEvent are
// reference-counted heap objects, lists hold references, clones are shallow,
// forwarding passes the SAME object, chunks link objects through their `next`
// field. That reproduces the aliasing effects the reference relies on
// (SURVEY.md Appendix A.7).
//
// Reference files restated (paths relative to
// modules/siddhi-core/src/main/java/io/siddhi/core/):
//   query/input/stream/state/StreamPreStateProcessor.java      -> StreamPre
//   query/input/stream/state/StreamPostStateProcessor.java     -> StreamPost
//   query/input/stream/state/CountPreStateProcessor.java       -> CountPre
//   query/input/stream/state/CountPostStateProcessor.java      -> CountPost
//   query/input/stream/state/LogicalPreStateProcessor.java     -> LogicalPre
//   query/input/stream/state/LogicalPostStateProcessor.java    -> LogicalPost
//   query/input/stream/state/AbsentStreamPreStateProcessor.java-> AbsentPre
//   query/input/stream/state/AbsentStreamPostStateProcessor.java-> AbsentPost
//   query/input/stream/state/runtime/*.java                     -> Inner*
//   query/input/stream/state/receiver/*.java,
//   query/input/{Single,Multi,StateMulti}ProcessStreamReceiver  -> Receiver
//   event/ComplexEventChunk.java                                -> Chunk
//   event/state/StateEvent.java, StateEventCloner.java,
//   event/stream/StreamEventCloner.java                         -> StateEvent/StreamEvent
//   util/snapshot/state/Partition{Sync,}StateHolder.java,
//   util/snapshot/state/SingleSyncStateHolder.java              -> Holder
//   partition/PartitionStreamReceiver.java:176-272,
//   partition/PartitionRuntimeImpl.java:346-364                 -> App::send / initPartition
//   query/selector/QuerySelector.java:76-313,
//   query/selector/attribute/aggregator/{Sum,Avg,Count,Max,Min}*-> Selector
//   query/output/ratelimit/OutputRateLimiter.java:63-106        -> Selector::sendToCallBacks
//   executor/condition/**, executor/math/**,
//   executor/VariableExpressionExecutor.java,
//   executor/function/IfThenElseFunctionExecutor.java           -> eval()
//   util/Scheduler.java:74-206, util/timestamp/TimestampGeneratorImpl.java -> Scheduler
//   java.util.HashMap iteration order of PartitionStateHolder.states    -> jhashmap.h
//   util/parser/StateInputStreamParser.java:76-408               -> QueryRT::parse
#include "refcpu.h"
#include "jhashmap.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

namespace ref {

// ---------------------------------------------------------------- refcounting
struct RC {
    int rc_ = 0;
};
template <class T>
class Ref {
   public:
    Ref() : p_(nullptr) {}
    Ref(T* p) : p_(p) { inc(); }
    Ref(const Ref& o) : p_(o.p_) { inc(); }
    Ref(Ref&& o) noexcept : p_(o.p_) { o.p_ = nullptr; }
    ~Ref() { dec(); }
    Ref& operator=(const Ref& o) {
        if (o.p_ != p_) {
            T* old = p_;
            p_ = o.p_;
            inc();
            if (old && --old->rc_ == 0) delete old;
        }
        return *this;
    }
    Ref& operator=(Ref&& o) noexcept {
        if (this != &o) {
            T* old = p_;
            p_ = o.p_;
            o.p_ = nullptr;
            if (old && --old->rc_ == 0) delete old;
        }
        return *this;
    }
    T* get() const { return p_; }
    T* operator->() const { return p_; }
    T& operator*() const { return *p_; }
    explicit operator bool() const { return p_ != nullptr; }
    bool operator==(const Ref& o) const { return p_ == o.p_; }
    bool operator!=(const Ref& o) const { return p_ != o.p_; }

   private:
    void inc() {
        if (p_) ++p_->rc_;
    }
    void dec() {
        if (p_ && --p_->rc_ == 0) delete p_;
        p_ = nullptr;
    }
    T* p_;
};

enum EvType { CURRENT = 0, EXPIRED = 1, TIMER = 2, RESET = 3 };

struct Val {
    int64_t b = 0;
    int8_t t = SH_T_OBJECT;
    bool null = true;
};

// Input event data (immutable once built; shared by every StreamEvent copy,
// StreamEventCloner.java:48-66 copies the data arrays whose elements are immutable).
struct Row : RC {
    int64_t ts;
    uint64_t seq;
    int stream;
    std::vector<int64_t> v;
    std::vector<uint8_t> nul;
};

struct StreamEvent : RC {
    int64_t ts = -1;
    EvType type = CURRENT;
    Ref<Row> row;
    Ref<StreamEvent> next;
    // long chains (count states) are released iteratively, not recursively
    ~StreamEvent() {
        Ref<StreamEvent> n = std::move(next);
        while (n && n->rc_ == 1) {
            Ref<StreamEvent> nn = std::move(n->next);
            n = std::move(nn);
        }
    }
};

struct StateEvent : RC {
    std::vector<Ref<StreamEvent>> ev;  // streamEvents[]
    Ref<StateEvent> next;              // ComplexEvent.next (chunk linkage)
    int64_t ts = -1;
    EvType type = CURRENT;
    std::vector<Val> out;              // outputData
    int64_t id = 0;
    uint64_t sel_seq = 0;              // oracle bookkeeping: trigger seq at selection
    StateEvent(int nslots, int nout) : ev(nslots), out(nout) {}
    ~StateEvent() {
        Ref<StateEvent> n = std::move(next);
        while (n && n->rc_ == 1) {
            Ref<StateEvent> nn = std::move(n->next);
            n = std::move(nn);
        }
    }
};

// ComplexEventChunk<E> semantics (event/ComplexEventChunk.java:32-282)
template <class E>
struct Chunk {
    Ref<E> first, prevToLastReturned, lastReturned, last;
    Chunk() {}
    Chunk(const Ref<E>& f, const Ref<E>& l) : first(f), last(l) {}
    static Ref<E> lastEvent(const Ref<E>& evs) {
        Ref<E> le = evs;
        while (le && le->next && le->next != evs) le = le->next;
        if (le && le->next == evs) le->next = Ref<E>();  // detach loop
        return le;
    }
    void add(const Ref<E>& evs) {
        if (!first) {
            first = evs;
        } else {
            last->next = evs;
        }
        last = lastEvent(evs);
    }
    bool hasNext() const {
        if (lastReturned) return (bool)lastReturned->next;
        if (prevToLastReturned) return (bool)prevToLastReturned->next;
        return (bool)first;
    }
    Ref<E> next() {
        Ref<E> r;
        if (lastReturned) {
            r = lastReturned->next;
            prevToLastReturned = lastReturned;
        } else if (prevToLastReturned) {
            r = prevToLastReturned->next;
        } else {
            r = first;
        }
        lastReturned = r;
        return r;
    }
    void remove() {
        if (prevToLastReturned) {
            prevToLastReturned->next = lastReturned->next;
        } else {
            first = lastReturned->next;
            if (!first) last = Ref<E>();
        }
        lastReturned->next = Ref<E>();
        lastReturned = Ref<E>();
    }
    void clear() {
        prevToLastReturned = Ref<E>();
        lastReturned = Ref<E>();
        first = Ref<E>();
        last = Ref<E>();
    }
    void reset() {
        prevToLastReturned = Ref<E>();
        lastReturned = Ref<E>();
    }
};

using SE = Ref<StateEvent>;
using SList = std::list<SE>;

struct App;
struct QueryRT;

// The partition flow key (SiddhiAppContext.startPartitionFlow thread-local).
struct Flow {
    int64_t key = INT64_MIN;  // INT64_MIN: not in a partition flow
};

// -------------------------------------------------------------- state holders
// PartitionSyncStateHolder / PartitionStateHolder (destroy on return when
// canDestroy and use count drops to 0) vs SingleSyncStateHolder (never).
struct StateBase {
    int use = 0;
    virtual ~StateBase() {}
    virtual bool canDestroy() { return false; }
};

template <class S>
struct Holder {
    App* app = nullptr;
    bool partitioned = false;
    std::function<S*()> factory;
    S* single = nullptr;
    std::unordered_map<int64_t, S*> states;
    int64_t ckey = INT64_MIN;  // one-entry lookup cache (same semantics as the map)
    S* cst = nullptr;
    // PartitionStateHolder.states as a java.util.HashMap (iteration order), kept
    // only where the order is observable (the Scheduler's holder)
    JHashMap* order = nullptr;
    S* get();
    void ret(S* s);
    ~Holder() {
        delete single;
        for (auto& kv : states) delete kv.second;
    }
};

// ---------------------------------------------------------------- processors
struct Proc {
    virtual ~Proc() {}
    virtual void process(Chunk<StateEvent>& c) = 0;
    Proc* nextProc = nullptr;  // Processor.getNextProcessor
    virtual void setToLast(Proc* p) {
        if (!nextProc)
            nextProc = p;
        else
            nextProc->setToLast(p);
    }
};

struct Selector;
struct StreamPost;
struct CountPre;

enum PreKind { K_STREAM, K_COUNT, K_LOGICAL, K_ABSENT, K_ABSENT_LOGICAL };

struct PreState : StateBase {
    Chunk<StateEvent> cur;  // currentStateEventChunk
    SList pending;          // pendingStateEventList
    SList nae;              // newAndEveryStateEventList
    bool changed = false;   // stateChanged
    bool initialized = false;
    bool started = false;
    bool canDestroy() override {
        return !cur.first && pending.empty() && nae.empty() && !initialized;
    }
};
struct CountPreState : PreState {
    bool success = false;     // successCondition
    bool startReset = false;  // startStateReset
};
struct AbsentPreState : PreState {
    int64_t lastScheduled = 0;  // lastScheduledTime
    bool active = true;
};

struct StreamPre : Proc {
    QueryRT* q = nullptr;
    PreKind kind = K_STREAM;
    int stateId = 0;
    bool isStart = false;
    int stateType = SH_PATTERN;
    int64_t within = -1;
    std::vector<int> startIds;
    StreamPre* withinEvery = nullptr;
    StreamPost* thisPost = nullptr;
    StreamPost* thisLast = nullptr;
    Holder<PreState> holder;

    void process(Chunk<StateEvent>&) override { abort(); }
    virtual ~StreamPre() {}
    virtual PreState* newState() { return new PreState(); }

    bool isExpired(StateEvent* se, int64_t now);
    void processSE(const SE& se);           // protected process(StateEvent)
    void init();
    void addState(const SE& se);
    virtual void addStateImpl(const SE& se, PreState* st);
    virtual void addEveryState(const SE& se);
    void stateChanged();
    virtual void resetState();
    virtual void updateState();
    virtual void expireEvents(int64_t ts);
    virtual Chunk<StateEvent> processAndReturn(const Ref<StreamEvent>& sev);
    virtual bool removeOnNoStateChange() { return stateType == SH_SEQUENCE; }
    SList* pendingList();  // getPendingStateEventList (state returned before use)
};

struct StreamPost : Proc {
    StreamPre* nextPre = nullptr;
    StreamPre* nextEveryPre = nullptr;
    StreamPre* thisPre = nullptr;
    int stateId = 0;
    CountPre* callbackPre = nullptr;
    bool returned = false;  // isEventReturned
    void process(Chunk<StateEvent>& c) override {
        c.reset();
        if (c.hasNext()) {
            SE se = c.next();
            processSE(se, c);
        }
        c.clear();
    }
    virtual void processSE(const SE& se, Chunk<StateEvent>& c);
    virtual void setNextStatePre(StreamPre* p) { nextPre = p; }
    virtual void setNextEveryStatePre(StreamPre* p) { nextEveryPre = p; }
};

struct CountPost;
struct CountPre : StreamPre {
    int minCount, maxCount;
    CountPost* countPost = nullptr;
    int resetDepth = 0;
    CountPre(int mn, int mx) : minCount(mn), maxCount(mx) { kind = K_COUNT; }
    PreState* newState() override { return new CountPreState(); }
    Chunk<StateEvent> processAndReturn(const Ref<StreamEvent>& sev) override;
    void successCondition();
    void addStateImpl(const SE& se, PreState* st) override;
    void addEveryState(const SE& se) override;
    void startStateReset();
    void updateState() override;
};

struct CountPost : StreamPost {
    int minCount, maxCount;
    CountPost(int mn, int mx) : minCount(mn), maxCount(mx) {}
    void processSE(const SE& se, Chunk<StateEvent>& c) override;
    void processMinCountReached(const SE& se, Chunk<StateEvent>& c);
    void setNextStatePre(StreamPre* p) override;
};

struct LogicalPre : StreamPre {
    int logicalType;  // SH_E_LOGICAL_AND / OR
    LogicalPre* partner = nullptr;
    explicit LogicalPre(int lt) : logicalType(lt) { kind = K_LOGICAL; }
    void addStateImpl(const SE& se, PreState* st) override;
    void addEveryState(const SE& se) override;
    void resetState() override;
    void updateState() override;
    Chunk<StateEvent> processAndReturn(const Ref<StreamEvent>& sev) override;
    void moveAllNaeToPending();
    bool isNaeEmpty();
    void addToNae(const SE& se);
    virtual bool partnerCanProceed(StateEvent*) { return true; }
};

struct LogicalPost : StreamPost {
    int type;
    LogicalPre* partnerPre = nullptr;
    LogicalPost* partnerPost = nullptr;
    explicit LogicalPost(int t) : type(t) {}
    void processSE(const SE& se, Chunk<StateEvent>& c) override;
    void setNextStatePre(StreamPre* p) override {
        nextPre = p;
        partnerPost->nextPre = p;
    }
    void setNextEveryStatePre(StreamPre* p) override {
        nextEveryPre = p;
        partnerPost->nextEveryPre = p;
    }
};

// --------------------------------------------------------------- scheduler
// util/Scheduler.java (playback / event-time semantics): per partition-key
// FIFO queue of notify times, head-peeked; due states collected through a
// TreeMultimap whose value comparator is always 0 (one state per due time).
struct AbsentPre;
struct SchedState : StateBase {
    std::list<int64_t> toNotify;  // toNotifyQueue (FIFO)
    bool canDestroy() override { return toNotify.empty(); }
};

struct Scheduler {
    App* app = nullptr;
    // EntryValveProcessor -> the absent pre-processor's process(TIMER chunk)
    std::function<void(int64_t)> target;
    Holder<SchedState> holder;
    // PartitionStateHolder.states in java.util.HashMap order: onTimeChange walks
    // it and keeps the first state per due time (Scheduler.java:77-86)
    JHashMap order;
    void notifyAt(int64_t t);
    void onTimeChange(int64_t now);
    void sendTimerEvents(SchedState* st, int64_t now);
    // wall-clock mode (Scheduler.EventCaller): earliest queued notify time, and
    // every state due at `now` fired on its own (no TreeMultimap collapse)
    int64_t nextDue() const;
    void fireAllDue(int64_t now);
};

struct AbsentPre : StreamPre {
    int64_t waitingTime;
    Scheduler* sched = nullptr;
    explicit AbsentPre(int64_t w) : waitingTime(w) { kind = K_ABSENT; }
    PreState* newState() override { return new AbsentPreState(); }
    void updateLastArrivalTime(int64_t ts);
    void addStateImpl(const SE& se, PreState* st) override;
    void addEveryState(const SE& se) override;
    void resetState() override;
    void processTimer(int64_t now);  // process(ComplexEventChunk) with a TIMER event
    void sendEvent(const SE& se, AbsentPreState* st);
    Chunk<StateEvent> processAndReturn(const Ref<StreamEvent>& sev) override;
    bool removeOnNoStateChange() override { return false; }
    void partitionCreated();
};

struct AbsentPost : StreamPost {
    void processSE(const SE& se, Chunk<StateEvent>& c) override;
};

// AbsentLogicalPreStateProcessor.java:65-420 / AbsentLogicalPostStateProcessor.java:37-49
struct LogicalAbsentState : PreState {
    int64_t lastArrivalTime = 0;
    bool active = true;
    bool canDestroy() override { return PreState::canDestroy() && lastArrivalTime == 0; }
};
struct AbsentLogicalPre : LogicalPre {
    int64_t waitingTime;
    Scheduler* sched = nullptr;
    AbsentLogicalPre(int lt, int64_t w) : LogicalPre(lt), waitingTime(w) { kind = K_ABSENT_LOGICAL; }
    PreState* newState() override { return new LogicalAbsentState(); }
    void updateLastArrivalTime(int64_t ts);
    void addStateImpl(const SE& se, PreState* st) override;
    void addEveryState(const SE& se) override;
    void processTimer(int64_t t);  // process(ComplexEventChunk) with a TIMER event
    bool waitingTimePassed(int64_t now, StateEvent* se);
    void sendEvent(const SE& se, LogicalAbsentState* st);
    void setActive(bool a);
    Chunk<StateEvent> processAndReturn(const Ref<StreamEvent>& sev) override;
    void partitionCreated();
    bool partnerCanProceed(StateEvent* se) override;
};
struct AbsentLogicalPost : LogicalPost {
    explicit AbsentLogicalPost(int t) : LogicalPost(t) {}
    void processSE(const SE& se, Chunk<StateEvent>& c) override;
};

// --------------------------------------------------------------- selector
struct AggState : StateBase {
    std::vector<double> dsum;
    std::vector<int64_t> lsum;
    std::vector<int64_t> cnt;
    std::vector<Val> mx;
};

struct Selector : Proc {
    QueryRT* q = nullptr;
    bool containsAggregator = false;
    std::unordered_map<int64_t, AggState*> agg;  // per partition flow key
    // with `group by`: per (partition flow key, group key) -- SiddhiAppContext.startGroupByFlow
    // (QuerySelector.java:315-340) keys the aggregators' state holders by the group key
    std::map<std::pair<int64_t, std::vector<int64_t>>, AggState*> aggG;
    ~Selector() {
        for (auto& kv : agg) delete kv.second;
        for (auto& kv : aggG) delete kv.second;
    }
    void process(Chunk<StateEvent>& c) override;
    std::vector<int64_t> groupKey(StateEvent* se);
    void populate(StateEvent* se);
    bool having(StateEvent* se);
    int orderCompare(StateEvent* a, StateEvent* b);
    void orderChunk(Chunk<StateEvent>& c);
    void offsetChunk(Chunk<StateEvent>& c);
    void limitChunk(Chunk<StateEvent>& c);
    void rateProcess(Chunk<StateEvent>& c);
    std::unordered_map<int64_t, int32_t> rateCounter;  // RateLimiterState per partition flow
    std::unordered_map<int64_t, Chunk<StateEvent>> rateHeld;  // AllPerEvent: allComplexEventChunk per partition flow
    std::unordered_map<int64_t, int64_t> rateOutTime;         // FirstPerTime: RateLimiterState.outputTime (absent: null)
    void sendToCallBacks(Chunk<StateEvent>& c);
};

// ---------------------------------------------------------------- receivers
struct Receiver {
    QueryRT* q = nullptr;
    int stream = 0;
    bool multi = false;
    std::vector<StreamPre*> nextProcessors;  // Multi: slot-ordered; Single: [0]
    int processCount = 1;
    std::vector<int> eventSequence;
    std::vector<StreamPre*> forStream;       // stateProcessorsForStream
    Selector* querySelector = nullptr;
    void setNext(StreamPre* p);
    void stabilizeStates(int64_t ts);
    void receive(const std::vector<Ref<Row>>& rows);
};

// -------------------------------------------------------------- inner runtimes
struct Inner {
    StreamPre* first = nullptr;
    StreamPost* last = nullptr;
    std::vector<std::pair<Receiver*, StreamPre*>> ssr;  // singleStreamRuntimeList
    virtual ~Inner() {}
    virtual void setQuerySelector(Proc* sel) { last->nextProc = sel; }
    virtual void setup() {
        ssr[0].first->setNext(first);
        ssr[0].first->forStream.push_back(first);
    }
    virtual void init() { first->init(); }
    virtual void reset() { first->resetState(); }
    virtual void update() { first->updateState(); }
};
struct NextInner : Inner {
    Inner *cur, *nxt;
    NextInner(Inner* c, Inner* n) : cur(c), nxt(n) {}
    void setQuerySelector(Proc* sel) override { nxt->setQuerySelector(sel); }
    void setup() override {
        cur->setup();
        nxt->setup();
    }
    void init() override {
        cur->init();
        nxt->init();
    }
    void reset() override {
        nxt->reset();
        cur->reset();
    }
    void update() override {
        cur->update();
        nxt->update();
    }
};
struct EveryInner : Inner {  // reset/update inherited: first processor only
    Inner* in;
    explicit EveryInner(Inner* i) : in(i) {}
    void setQuerySelector(Proc* sel) override { in->setQuerySelector(sel); }
    void setup() override { in->setup(); }
    void init() override { in->init(); }
};
struct LogicalInner : Inner {
    Inner *in1, *in2;
    LogicalInner(Inner* a, Inner* b) : in1(a), in2(b) {}
    void setQuerySelector(Proc* sel) override {
        in2->setQuerySelector(sel);
        in1->setQuerySelector(sel);
    }
    void setup() override {
        in2->setup();
        in1->setup();
    }
    void init() override {
        in2->init();
        in1->init();
    }
    void reset() override { in2->reset(); }
    void update() override { in2->update(); }
};

struct FilterProc : Proc {
    QueryRT* q;
    int expr;
    FilterProc(QueryRT* qq, int e) : q(qq), expr(e) {}
    void process(Chunk<StateEvent>& c) override;
};

// ------------------------------------------------------------------- query
struct QueryRT {
    App* app = nullptr;
    int index = 0;
    sh_query_desc d;
    std::vector<sh_state_elem> elems;
    std::vector<sh_expr> exprs;
    std::vector<sh_output_attr> outs;
    int nslots = 0;
    int partition = -1;
    std::vector<std::unique_ptr<Proc>> owned;
    std::vector<std::unique_ptr<Inner>> ownedInner;
    std::vector<std::unique_ptr<Scheduler>> scheds;
    std::map<int, std::unique_ptr<Receiver>> receivers;  // by stream
    std::vector<StreamPre*> pres;         // preStateProcessors (parse order)
    std::vector<StreamPre*> startupPres;  // startupPreStateProcessors
    Inner* root = nullptr;
    Selector* selector = nullptr;
    int slotCounter = 0;
    std::string err;

    template <class T, class... A>
    T* own(A&&... a) {
        T* p = new T(std::forward<A>(a)...);
        owned.emplace_back(p);
        return p;
    }
    template <class T, class... A>
    T* ownI(A&&... a) {
        T* p = new T(std::forward<A>(a)...);
        ownedInner.emplace_back(p);
        return p;
    }
    SE newStateEvent() { return SE(new StateEvent(nslots, (int)outs.size())); }
    SE copyStateEvent(const SE& s) {
        SE n = newStateEvent();
        n->out = s->out;
        n->ev = s->ev;
        n->type = s->type;
        n->ts = s->ts;
        n->id = s->id;
        return n;
    }
    static Ref<StreamEvent> copyStreamEvent(const Ref<StreamEvent>& s) {
        Ref<StreamEvent> n(new StreamEvent());
        n->row = s->row;
        n->type = s->type;
        n->ts = s->ts;
        return n;
    }
    bool build();
    Inner* parse(int e, StreamPre* pre, StreamPost* post, std::vector<StreamPre*>& list, bool isStart);
    void initPartition();
    Val eval(int e, StateEvent* se);
};

struct OutRow {
    int32_t query;
    uint64_t seq;
    int64_t ts;
    std::vector<Val> v;
    int32_t group;
};

// Multi receivers defer callbacks through a thread-local ReturnEventHolder
// (MultiProcessStreamReceiver.java:42,306-315).
struct ReturnHolder {
    Chunk<StateEvent> chunk;
    bool has = false;
    Selector* sel = nullptr;
};

struct PartitionRT {
    std::vector<QueryRT*> queries;
    std::set<int64_t> seen;  // PartitionState.partitionKeys
};

struct App {
    sh_app_desc d;
    std::vector<std::vector<int32_t>> streamTypes;
    std::vector<std::unique_ptr<QueryRT>> queries;
    std::vector<PartitionRT> partitions;
    std::vector<uint8_t> partStreams;
    // junction subscribers per stream: (query index) or (-1 - partition)
    std::vector<std::vector<int>> subs;
    Flow flow;
    ReturnHolder* holder = nullptr;
    uint64_t curSeq = 0;
    uint64_t nextSeq = 0;  // sequence number of the next input event
    int32_t cbGroup = 0;
    int64_t clock = 0;  // TimestampGeneratorImpl current time (playback)
    std::vector<OutRow> out;
    // List values of SH_OP_MULTI_VAR outputs (a row holds the list's index)
    std::vector<std::vector<int64_t>> listV;
    std::vector<std::vector<uint8_t>> listN;
    std::vector<StateBase*> zombies;  // destroyed states still referenced in-frame
    std::vector<Scheduler*> schedulers;
    std::string err;
    // attr.toString() of every partition key id (ValuePartitionExecutor.java:34-40),
    // UTF-16; an id never registered reads as its decimal digits
    std::vector<std::u16string> keyStr;
    std::vector<uint8_t> keyHas;
    std::vector<int32_t> keyHashes;  // String.hashCode cache (valid where keyHas)
    std::u16string keyString(int64_t k) const {
        if (k >= 0 && k < (int64_t)keyStr.size() && keyHas[k]) return keyStr[k];
        std::string d = std::to_string(k);
        return std::u16string(d.begin(), d.end());
    }
    int32_t keyHash(int64_t k) const {
        if (k >= 0 && k < (int64_t)keyHas.size() && keyHas[k]) return keyHashes[k];
        const std::u16string s = keyString(k);
        return java_string_hash((const uint16_t*)s.data(), (int64_t)s.size());
    }
    int keyCompare(int64_t a, int64_t b) const {
        const std::u16string x = keyString(a), y = keyString(b);
        return java_string_compare((const uint16_t*)x.data(), (int64_t)x.size(), (const uint16_t*)y.data(),
                                   (int64_t)y.size());
    }
    ~App() {
        for (auto* z : zombies) delete z;
    }
    void flushZombies() {
        for (auto* z : zombies) delete z;
        zombies.clear();
    }
};

template <class S>
S* Holder<S>::get() {
    if (!partitioned) {
        if (!single) single = factory();
        return single;
    }
    const int64_t key = app->flow.key;
    if (order) order->computeIfAbsent(key);  // states.computeIfAbsent(partitionFlowId, ...)
    if (cst && ckey == key) {
        cst->use++;
        return cst;
    }
    S*& p = states[key];
    if (!p) p = factory();
    p->use++;
    ckey = key;
    cst = p;
    return p;
}
template <class S>
void Holder<S>::ret(S* s) {
    if (!partitioned) return;
    s->use--;
    if (s->use == 0 && s->canDestroy()) {
        auto it = states.find(app->flow.key);
        if (it != states.end() && it->second == s) states.erase(it);
        if (order) order->remove(app->flow.key, true);  // removeState -> HashMap.remove
        if (cst == s) cst = nullptr;
        app->zombies.push_back(s);
    }
}

// ----------------------------------------------------------------- eval
static inline float f32(int64_t b) {
    float f;
    uint32_t u = (uint32_t)b;
    memcpy(&f, &u, 4);
    return f;
}
static inline double f64(int64_t b) {
    double d;
    memcpy(&d, &b, 8);
    return d;
}
static inline int64_t bf32(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (int64_t)u;
}
static inline int64_t bf64(double d) {
    int64_t b;
    memcpy(&b, &d, 8);
    return b;
}
static inline int32_t i32(int64_t b) { return (int32_t)b; }

// Number.xxxValue() conversions of a typed raw value
static double asD(const Val& v) {
    switch (v.t) {
        case SH_T_INT: return (double)i32(v.b);
        case SH_T_LONG: return (double)v.b;
        case SH_T_FLOAT: return (double)f32(v.b);
        case SH_T_DOUBLE: return f64(v.b);
        default: return 0;
    }
}
static float asF(const Val& v) {
    switch (v.t) {
        case SH_T_INT: return (float)i32(v.b);
        case SH_T_LONG: return (float)v.b;
        case SH_T_FLOAT: return f32(v.b);
        case SH_T_DOUBLE: return (float)f64(v.b);
        default: return 0;
    }
}
static int64_t asL(const Val& v) {
    switch (v.t) {
        case SH_T_INT: return (int64_t)i32(v.b);
        case SH_T_LONG: return v.b;
        case SH_T_FLOAT: {  // Java (long) cast semantics
            float f = f32(v.b);
            if (f != f) return 0;
            if (f >= 9.2233720368547758e18f) return INT64_MAX;
            if (f <= -9.2233720368547758e18f) return INT64_MIN;
            return (int64_t)f;
        }
        case SH_T_DOUBLE: {
            double d = f64(v.b);
            if (d != d) return 0;
            if (d >= 9.2233720368547758e18) return INT64_MAX;
            if (d <= -9.2233720368547758e18) return INT64_MIN;
            return (int64_t)d;
        }
        default: return 0;
    }
}
static int32_t asI(const Val& v) {
    switch (v.t) {
        case SH_T_INT: return i32(v.b);
        case SH_T_LONG: return (int32_t)(uint32_t)(uint64_t)v.b;
        case SH_T_FLOAT: {
            float f = f32(v.b);
            if (f != f) return 0;
            if (f >= 2147483648.0f) return INT32_MAX;
            if (f <= -2147483648.0f) return INT32_MIN;
            return (int32_t)f;
        }
        case SH_T_DOUBLE: {
            double d = f64(v.b);
            if (d != d) return 0;
            if (d >= 2147483648.0) return INT32_MAX;
            if (d <= -2147483648.0) return INT32_MIN;
            return (int32_t)d;
        }
        default: return 0;
    }
}
static int rank(int t) {
    switch (t) {
        case SH_T_INT: return 0;
        case SH_T_LONG: return 1;
        case SH_T_FLOAT: return 2;
        case SH_T_DOUBLE: return 3;
        default: return -1;
    }
}

static Val mkBool(bool b) {
    Val v;
    v.t = SH_T_BOOL;
    v.null = false;
    v.b = b ? 1 : 0;
    return v;
}
static Val mkNull(int t) {
    Val v;
    v.t = (int8_t)t;
    v.null = true;
    return v;
}

// compare executors: Java binary numeric promotion of the unboxed operands,
// except ==/!= on (Float,Long)/(Long,Float) which compare as double
// (executor/condition/compare/equal/EqualCompareConditionExpressionExecutorFloatLong.java).
static bool cmp(int op, const Val& l, const Val& r) {
    if (l.t == SH_T_STRING || r.t == SH_T_STRING) {
        bool eq = l.b == r.b;
        return op == SH_OP_EQ ? eq : !eq;
    }
    if (l.t == SH_T_BOOL || r.t == SH_T_BOOL) {
        bool eq = (l.b != 0) == (r.b != 0);
        return op == SH_OP_EQ ? eq : !eq;
    }
    int rk = std::max(rank(l.t), rank(r.t));
    bool fl = (l.t == SH_T_FLOAT && r.t == SH_T_LONG) || (l.t == SH_T_LONG && r.t == SH_T_FLOAT);
    if ((op == SH_OP_EQ || op == SH_OP_NE) && fl) rk = 3;
    switch (rk) {
        case 3: {
            double a = asD(l), b = asD(r);
            switch (op) {
                case SH_OP_EQ: return a == b;
                case SH_OP_NE: return a != b;
                case SH_OP_GT: return a > b;
                case SH_OP_GE: return a >= b;
                case SH_OP_LT: return a < b;
                default: return a <= b;
            }
        }
        case 2: {
            float a = asF(l), b = asF(r);
            switch (op) {
                case SH_OP_EQ: return a == b;
                case SH_OP_NE: return a != b;
                case SH_OP_GT: return a > b;
                case SH_OP_GE: return a >= b;
                case SH_OP_LT: return a < b;
                default: return a <= b;
            }
        }
        case 1: {
            int64_t a = asL(l), b = asL(r);
            switch (op) {
                case SH_OP_EQ: return a == b;
                case SH_OP_NE: return a != b;
                case SH_OP_GT: return a > b;
                case SH_OP_GE: return a >= b;
                case SH_OP_LT: return a < b;
                default: return a <= b;
            }
        }
        default: {
            int32_t a = asI(l), b = asI(r);
            switch (op) {
                case SH_OP_EQ: return a == b;
                case SH_OP_NE: return a != b;
                case SH_OP_GT: return a > b;
                case SH_OP_GE: return a >= b;
                case SH_OP_LT: return a < b;
                default: return a <= b;
            }
        }
    }
}

// math executors (executor/math/**): result type chosen at parse time;
// integral and floating divide/mod by zero yield null.
static Val arith(int op, int rt, const Val& l, const Val& r) {
    if (l.null || r.null) return mkNull(rt);
    Val o;
    o.t = (int8_t)rt;
    o.null = false;
    switch (rt) {
        case SH_T_INT: {
            uint32_t a = (uint32_t)asI(l), b = (uint32_t)asI(r);
            int32_t sa = (int32_t)a, sb = (int32_t)b;
            int32_t res = 0;
            switch (op) {
                case SH_OP_ADD: res = (int32_t)(a + b); break;
                case SH_OP_SUB: res = (int32_t)(a - b); break;
                case SH_OP_MUL: res = (int32_t)(a * b); break;
                case SH_OP_DIV:
                    if (sb == 0) return mkNull(rt);
                    res = (sa == INT32_MIN && sb == -1) ? INT32_MIN : sa / sb;
                    break;
                default:
                    if (sb == 0) return mkNull(rt);
                    res = (sb == -1) ? 0 : sa % sb;
            }
            o.b = res;
            return o;
        }
        case SH_T_LONG: {
            uint64_t a = (uint64_t)asL(l), b = (uint64_t)asL(r);
            int64_t sa = (int64_t)a, sb = (int64_t)b;
            int64_t res = 0;
            switch (op) {
                case SH_OP_ADD: res = (int64_t)(a + b); break;
                case SH_OP_SUB: res = (int64_t)(a - b); break;
                case SH_OP_MUL: res = (int64_t)(a * b); break;
                case SH_OP_DIV:
                    if (sb == 0) return mkNull(rt);
                    res = (sa == INT64_MIN && sb == -1) ? INT64_MIN : sa / sb;
                    break;
                default:
                    if (sb == 0) return mkNull(rt);
                    res = (sb == -1) ? 0 : sa % sb;
            }
            o.b = res;
            return o;
        }
        case SH_T_FLOAT: {
            float a = asF(l), b = asF(r), res = 0;
            switch (op) {
                case SH_OP_ADD: res = a + b; break;
                case SH_OP_SUB: res = a - b; break;
                case SH_OP_MUL: res = a * b; break;
                case SH_OP_DIV:
                    if (b == 0.0f) return mkNull(rt);
                    res = a / b;
                    break;
                default:
                    if (b == 0.0f) return mkNull(rt);
                    res = fmodf(a, b);
            }
            o.b = bf32(res);
            return o;
        }
        default: {
            double a = asD(l), b = asD(r), res = 0;
            switch (op) {
                case SH_OP_ADD: res = a + b; break;
                case SH_OP_SUB: res = a - b; break;
                case SH_OP_MUL: res = a * b; break;
                case SH_OP_DIV:
                    if (b == 0.0) return mkNull(rt);
                    res = a / b;
                    break;
                default:
                    if (b == 0.0) return mkNull(rt);
                    res = fmod(a, b);
            }
            o.b = bf64(res);
            return o;
        }
    }
}

// StateEvent.getStreamEvent(int[] position), event/state/StateEvent.java:138-182
static StreamEvent* chainAt(StateEvent* se, int slot, int idx) {
    if (slot < 0 || slot >= (int)se->ev.size()) return nullptr;
    StreamEvent* s = se->ev[slot].get();
    if (!s) return nullptr;
    if (idx >= 0) {
        for (int i = 1; i <= idx; i++) {
            s = s->next.get();
            if (!s) return nullptr;
        }
    } else if (idx == SH_CHAIN_CURRENT) {
        while (s->next) s = s->next.get();
    } else if (idx == SH_CHAIN_LAST) {
        if (!s->next) return nullptr;
        while (s->next->next) s = s->next.get();
    } else {
        std::vector<StreamEvent*> l;
        while (s) {
            l.push_back(s);
            s = s->next.get();
        }
        int k = (int)l.size() + idx;
        if (k < 0) return nullptr;
        s = l[k];
    }
    return s;
}

Val QueryRT::eval(int e, StateEvent* se) {
    const sh_expr& x = exprs[e];
    switch (x.op) {
        case SH_OP_CONST: {
            Val v;
            v.t = (int8_t)x.type;
            v.null = x.is_null != 0;
            v.b = x.cval;
            return v;
        }
        case SH_OP_VAR: {
            StreamEvent* s = chainAt(se, x.slot, x.chain);
            if (!s) return mkNull(x.type);
            Val v;
            v.t = (int8_t)x.type;
            v.b = s->row->v[x.attr];
            v.null = s->row->nul[x.attr] != 0;
            return v;
        }
        case SH_OP_MULTI_VAR: {
            // MultiValueVariableFunctionExecutor.execute (MultiValueVariableFunctionExecutor.java:62-70):
            // getStreamEvent(position), then the attribute of it and every later event of the chain
            std::vector<int64_t> lv;
            std::vector<uint8_t> ln;
            for (StreamEvent* s = chainAt(se, x.slot, x.chain); s; s = s->next.get()) {
                lv.push_back(s->row->v[x.attr]);
                ln.push_back(s->row->nul[x.attr] != 0);
            }
            Val v;
            v.t = SH_T_OBJECT;
            v.null = false;
            v.b = (int64_t)app->listV.size();
            app->listV.push_back(std::move(lv));
            app->listN.push_back(std::move(ln));
            return v;
        }
        case SH_OP_AND: {
            Val l = eval(x.lhs, se);
            if (!l.null && l.b) {
                Val r = eval(x.rhs, se);
                if (!r.null && r.b) return mkBool(true);
            }
            return mkBool(false);
        }
        case SH_OP_OR: {
            Val l = eval(x.lhs, se);
            if (!l.null && l.b) return mkBool(true);
            Val r = eval(x.rhs, se);
            if (!r.null && r.b) return mkBool(true);
            return mkBool(false);
        }
        case SH_OP_NOT: {
            Val l = eval(x.lhs, se);
            return mkBool(!(!l.null && l.b));
        }
        case SH_OP_BOOL_VAR: {
            Val l = eval(x.lhs, se);
            return mkBool(!l.null && l.b);
        }
        case SH_OP_OUTPUT: {
            // HAVING_STATE variable: the selected event's output data (outputData)
            if (x.attr < 0 || x.attr >= (int)se->out.size()) return mkNull(x.type);
            return se->out[x.attr];
        }
        case SH_OP_EQ:
        case SH_OP_NE:
        case SH_OP_GT:
        case SH_OP_GE:
        case SH_OP_LT:
        case SH_OP_LE: {
            Val l = eval(x.lhs, se);
            Val r = eval(x.rhs, se);
            if (l.null || r.null) return mkBool(false);
            return mkBool(cmp(x.op, l, r));
        }
        case SH_OP_ADD:
        case SH_OP_SUB:
        case SH_OP_MUL:
        case SH_OP_DIV:
        case SH_OP_MOD: {
            Val l = eval(x.lhs, se);
            Val r = eval(x.rhs, se);
            return arith(x.op, x.type, l, r);
        }
        case SH_OP_IS_NULL: {
            Val l = eval(x.lhs, se);
            return mkBool(l.null);
        }
        case SH_OP_IS_NULL_STREAM: {
            StreamEvent* s = chainAt(se, x.slot, x.chain);
            return mkBool(s == nullptr);
        }
        case SH_OP_IF_THEN_ELSE: {
            Val c = eval(x.lhs, se);
            bool cond = !c.null && c.b;
            Val r = cond ? eval(x.rhs, se) : eval(x.third, se);
            r.t = (int8_t)x.type;
            return r;
        }
    }
    return mkNull(x.type);
}

// ------------------------------------------------------------ filter proc
// query/processor/filter/FilterProcessor.java:48-61
void FilterProc::process(Chunk<StateEvent>& c) {
    c.reset();
    while (c.hasNext()) {
        SE ev = c.next();
        Val r = q->eval(expr, ev.get());
        if (r.null || !r.b) c.remove();
    }
    if (c.first) nextProc->process(c);
}

// ------------------------------------------------------------ StreamPre
// StreamPreStateProcessor.java:118-129
bool StreamPre::isExpired(StateEvent* se, int64_t now) {
    if (within != -1) {
        for (int sid : startIds) {
            StreamEvent* s = se->ev[sid].get();
            if (s && std::llabs(s->ts - now) > within) return true;
        }
    }
    return false;
}
// :131-142
void StreamPre::processSE(const SE& se) {
    PreState* st = holder.get();
    st->cur.add(se);
    st->cur.reset();
    st->changed = false;
    nextProc->process(st->cur);
    st->cur.reset();
    holder.ret(st);
}
static bool nextIsAbsent(StreamPost* p);
// :178-194
void StreamPre::init() {
    PreState* st = holder.get();
    if (isStart && (!st->initialized || thisPost->nextEveryPre != nullptr ||
                    (stateType == SH_SEQUENCE && nextIsAbsent(thisPost)))) {
        SE se = q->newStateEvent();
        addState(se);
        st->initialized = true;
    }
    holder.ret(st);
}
// :204-227
void StreamPre::addState(const SE& se) {
    PreState* st = holder.get();
    addStateImpl(se, st);
    holder.ret(st);
}
void StreamPre::addStateImpl(const SE& se, PreState* st) {
    if (stateType == SH_SEQUENCE) {
        if (st->nae.empty()) st->nae.push_back(se);
    } else {
        st->nae.push_back(se);
    }
}
// :229-247
void StreamPre::addEveryState(const SE& se) {
    SE c = q->copyStateEvent(se);
    c->type = CURRENT;
    for (int i = stateId; i < (int)c->ev.size(); i++) c->ev[i] = Ref<StreamEvent>();
    PreState* st = holder.get();
    st->nae.push_back(c);
    holder.ret(st);
}
void StreamPre::stateChanged() {
    PreState* st = holder.get();
    st->changed = true;
    holder.ret(st);
}
SList* StreamPre::pendingList() {
    PreState* st = holder.get();
    holder.ret(st);
    return &st->pending;  // may be a just-destroyed (zombie) state: empty list
}
// :287-305
void StreamPre::resetState() {
    PreState* st = holder.get();
    st->pending.clear();
    if (isStart && st->nae.empty()) {
        if (stateType == SH_SEQUENCE && thisPost->nextEveryPre == nullptr &&
            !thisPost->nextPre->pendingList()->empty()) {
            holder.ret(st);
            return;
        }
        init();
    }
    holder.ret(st);
}
static bool tsLess(const SE& a, const SE& b) {
    // eventTimeComparator, StreamPreStateProcessor.java:66-80 (-1 sorts last)
    int64_t x = a->ts, y = b->ts;
    if (x == -1) return false;
    if (y == -1) return true;
    return x < y;
}
// :307-323
void StreamPre::updateState() {
    PreState* st = holder.get();
    st->nae.sort(tsLess);  // std::list::sort is stable, like List.sort (TimSort)
    st->pending.splice(st->pending.end(), st->nae);
    holder.ret(st);
}
// :325-361
void StreamPre::expireEvents(int64_t ts) {
    PreState* st = holder.get();
    SE expired;
    for (auto it = st->pending.begin(); it != st->pending.end();) {
        SE se = *it;
        if (isExpired(se.get(), ts)) {
            it = st->pending.erase(it);
            if (se->type != EXPIRED) {
                se->type = EXPIRED;
                expired = se;
            }
        } else {
            break;
        }
    }
    for (auto it = st->nae.begin(); it != st->nae.end();) {
        SE se = *it;
        if (isExpired(se.get(), ts)) {
            it = st->nae.erase(it);
            if (se->type != EXPIRED) {
                se->type = EXPIRED;
                expired = se;
            }
        } else {
            ++it;
        }
    }
    if (expired && withinEvery) {
        withinEvery->addEveryState(expired);
        withinEvery->updateState();
    }
    holder.ret(st);
}
// :363-403
Chunk<StateEvent> StreamPre::processAndReturn(const Ref<StreamEvent>& sev) {
    Chunk<StateEvent> ret;
    PreState* st = holder.get();
    for (auto it = st->pending.begin(); it != st->pending.end();) {
        SE se = *it;
        se->ev[stateId] = QueryRT::copyStreamEvent(sev);
        processSE(se);
        if (thisLast->returned) {
            thisLast->returned = false;
            ret.add(se);
        }
        if (st->changed) {
            it = st->pending.erase(it);
        } else {
            if (stateType == SH_PATTERN) {
                se->ev[stateId] = Ref<StreamEvent>();
                ++it;
            } else {
                se->ev[stateId] = Ref<StreamEvent>();
                if (removeOnNoStateChange())
                    it = st->pending.erase(it);
                else
                    ++it;
                if (thisPost->callbackPre) thisPost->callbackPre->startStateReset();
            }
        }
    }
    holder.ret(st);
    return ret;
}

// ------------------------------------------------------------ StreamPost
// StreamPostStateProcessor.java:64-83
void StreamPost::processSE(const SE& se, Chunk<StateEvent>& c) {
    thisPre->stateChanged();
    StreamEvent* s = se->ev[stateId].get();
    se->ts = s->ts;
    if (nextProc) {
        c.reset();
        returned = true;
    }
    if (nextPre) nextPre->addState(se);
    if (nextEveryPre) nextEveryPre->addEveryState(se);
    if (callbackPre) callbackPre->startStateReset();
}
static bool nextIsAbsent(StreamPost* p) {
    return p->nextPre && (p->nextPre->kind == K_ABSENT || p->nextPre->kind == K_ABSENT_LOGICAL);
}

// ------------------------------------------------------------ CountPre
// CountPreStateProcessor.java:52-103
Chunk<StateEvent> CountPre::processAndReturn(const Ref<StreamEvent>& sev) {
    Chunk<StateEvent> ret;
    CountPreState* st = (CountPreState*)holder.get();
    for (auto it = st->pending.begin(); it != st->pending.end();) {
        SE se = *it;
        bool removed = false;
        for (int pos : {stateId + 1, stateId + 2}) {
            if ((int)se->ev.size() > pos && se->ev[pos]) {
                it = st->pending.erase(it);
                removed = true;
                break;
            }
        }
        if (removed) continue;
        // StateEvent.addEvent, StateEvent.java:212-222
        Ref<StreamEvent> ne = QueryRT::copyStreamEvent(sev);
        if (!se->ev[stateId]) {
            se->ev[stateId] = ne;
        } else {
            StreamEvent* t = se->ev[stateId].get();
            while (t->next) t = t->next.get();
            t->next = ne;
        }
        st->success = false;
        processSE(se);
        if (thisLast->returned) {
            thisLast->returned = false;
            ret.add(se);
        }
        bool erased = false;
        if (st->changed) {
            it = st->pending.erase(it);
            erased = true;
        }
        if (!st->success) {
            // StateEvent.removeLastEvent, StateEvent.java:224-236
            StreamEvent* t = se->ev[stateId].get();
            if (t) {
                bool done = false;
                while (t->next) {
                    if (!t->next->next) {
                        t->next = Ref<StreamEvent>();
                        done = true;
                        break;
                    }
                    t = t->next.get();
                }
                if (!done) se->ev[stateId] = Ref<StreamEvent>();
            }
            if (stateType == SH_SEQUENCE && !erased) {
                it = st->pending.erase(it);
                erased = true;
            }
        }
        if (!erased) ++it;
    }
    holder.ret(st);
    return ret;
}
void CountPre::successCondition() {
    CountPreState* st = (CountPreState*)holder.get();
    st->success = true;
    holder.ret(st);
}
// :114-138
void CountPre::addStateImpl(const SE& se, PreState* st) {
    if (stateType == SH_SEQUENCE) {
        if (st->nae.empty()) st->nae.push_back(se);
    } else {
        st->nae.push_back(se);
    }
    if (minCount == 0 && !se->ev[stateId]) {
        Chunk<StateEvent>& c = st->cur;
        c.clear();
        c.add(se);
        countPost->processMinCountReached(se, c);
        c.clear();
    }
}
void CountPre::addEveryState(const SE& se) { StreamPre::addEveryState(se); }
// :168-179
void CountPre::startStateReset() {
    CountPreState* st = (CountPreState*)holder.get();
    st->startReset = true;
    if (thisPost->callbackPre) {
        if (resetDepth < 64) {  // the reference recurses here; bound it
            resetDepth++;
            ((CountPre*)((StreamPost*)countPost)->thisPre)->startStateReset();
            resetDepth--;
        } else {
            q->err = "CountPreStateProcessor.startStateReset recursion";
        }
    }
    holder.ret(st);
}
// :181-193
void CountPre::updateState() {
    CountPreState* st = (CountPreState*)holder.get();
    if (st->startReset) {
        st->startReset = false;
        init();
    }
    StreamPre::updateState();
    holder.ret(st);
}

// ------------------------------------------------------------ CountPost
// CountPostStateProcessor.java:39-89
void CountPost::processSE(const SE& se, Chunk<StateEvent>& c) {
    StreamEvent* s = se->ev[stateId].get();
    int n = 1;
    while (s->next) {
        n++;
        s = s->next.get();
    }
    ((CountPre*)thisPre)->successCondition();
    se->ts = s->ts;
    if (n >= minCount) {
        if (thisPre->stateType == SH_SEQUENCE) {
            if (nextPre) nextPre->addState(se);
            if (n != maxCount) thisPre->addState(se);
        } else if (n == minCount) {
            processMinCountReached(se, c);
        }
        if (n == maxCount) thisPre->stateChanged();
    }
}
void CountPost::processMinCountReached(const SE& se, Chunk<StateEvent>& c) {
    if (nextProc) {
        thisPre->stateChanged();
        c.reset();
        returned = true;
    }
    if (nextPre) nextPre->addState(se);
    if (nextEveryPre) nextEveryPre->addEveryState(se);
}
void CountPost::setNextStatePre(StreamPre* p) {
    nextPre = p;
    if (thisPre->isStart && thisPre->stateType == SH_SEQUENCE && minCount == 0) {
        p->thisPost->callbackPre = (CountPre*)thisPre;
    }
}

// ------------------------------------------------------------ LogicalPre
// LogicalPreStateProcessor.java:43-201
void LogicalPre::addStateImpl(const SE& se, PreState* st) {
    if (isStart || stateType == SH_SEQUENCE) {
        if (st->nae.empty()) st->nae.push_back(se);
        if (partner && partner->isNaeEmpty()) partner->addToNae(se);
    } else {
        st->nae.push_back(se);
        if (partner) partner->addToNae(se);
    }
}
void LogicalPre::addEveryState(const SE& se) {
    SE c = q->copyStateEvent(se);
    c->type = CURRENT;
    c->ev[stateId] = Ref<StreamEvent>();
    for (int i = stateId; i < (int)c->ev.size(); i++) c->ev[i] = Ref<StreamEvent>();
    PreState* st = holder.get();
    st->nae.push_back(c);
    if (partner) {
        c->ev[partner->stateId] = Ref<StreamEvent>();
        partner->addToNae(c);
    }
    holder.ret(st);
}
void LogicalPre::resetState() {
    PreState* st = holder.get();
    if (logicalType == SH_E_LOGICAL_OR || st->pending.size() == partner->pendingList()->size()) {
        st->pending.clear();
        partner->pendingList()->clear();
        if (isStart && st->nae.empty()) {
            if (stateType == SH_SEQUENCE && thisPost->nextEveryPre == nullptr &&
                !thisPost->nextPre->pendingList()->empty()) {
                holder.ret(st);
                return;
            }
            init();
        }
    }
    holder.ret(st);
}
void LogicalPre::updateState() {
    PreState* st = holder.get();
    st->nae.sort(tsLess);
    st->pending.splice(st->pending.end(), st->nae);
    partner->moveAllNaeToPending();
    holder.ret(st);
}
Chunk<StateEvent> LogicalPre::processAndReturn(const Ref<StreamEvent>& sev) {
    Chunk<StateEvent> ret;
    PreState* st = holder.get();
    for (auto it = st->pending.begin(); it != st->pending.end();) {
        SE se = *it;
        if (logicalType == SH_E_LOGICAL_OR && se->ev[partner->stateId]) {
            it = st->pending.erase(it);
            continue;
        }
        se->ev[stateId] = QueryRT::copyStreamEvent(sev);
        processSE(se);
        if (thisLast->returned) {
            thisLast->returned = false;
            ret.add(se);
        }
        if (st->changed) {
            it = st->pending.erase(it);
        } else {
            se->ev[stateId] = Ref<StreamEvent>();
            if (stateType == SH_PATTERN)
                ++it;
            else
                it = st->pending.erase(it);
        }
    }
    holder.ret(st);
    return ret;
}
void LogicalPre::moveAllNaeToPending() {
    PreState* st = holder.get();
    st->nae.sort(tsLess);
    st->pending.splice(st->pending.end(), st->nae);
    holder.ret(st);
}
bool LogicalPre::isNaeEmpty() {
    PreState* st = holder.get();
    bool r = st->nae.empty();
    holder.ret(st);
    return r;
}
void LogicalPre::addToNae(const SE& se) {
    PreState* st = holder.get();
    st->nae.push_back(se);
    holder.ret(st);
}

// ------------------------------------------------------------ LogicalPost
// LogicalPostStateProcessor.java:59-87
void LogicalPost::processSE(const SE& se, Chunk<StateEvent>& c) {
    if (type == SH_E_LOGICAL_AND) {
        bool proceed;
        if (partnerPre->kind == K_ABSENT_LOGICAL)
            proceed = partnerPre->partnerCanProceed(se.get());
        else
            proceed = (bool)se->ev[partnerPre->stateId];
        if (proceed)
            StreamPost::processSE(se, c);
        else
            thisPre->stateChanged();
    } else {
        StreamPost::processSE(se, c);
        if (partnerPost->nextProc && thisPre->thisLast == partnerPost) partnerPost->returned = true;
    }
}

// ------------------------------------------------------------ Absent
// AbsentStreamPreStateProcessor.java:67-342 (event-time / playback semantics)
void AbsentPre::updateLastArrivalTime(int64_t ts) {
    AbsentPreState* st = (AbsentPreState*)holder.get();
    st->lastScheduled = ts + waitingTime;
    sched->notifyAt(st->lastScheduled);
    holder.ret(st);
}
void AbsentPre::addStateImpl(const SE& se, PreState* pst) {
    AbsentPreState* st = (AbsentPreState*)pst;
    if (!st->active) return;
    if (stateType == SH_SEQUENCE) {
        st->nae.clear();
        st->nae.push_back(se);
    } else {
        st->nae.push_back(se);
    }
    if (!isStart) {
        st->lastScheduled = se->ts + waitingTime;
        sched->notifyAt(st->lastScheduled);
    }
}
void AbsentPre::addEveryState(const SE& se) {
    AbsentPreState* st = (AbsentPreState*)holder.get();
    SE c = q->copyStateEvent(se);
    c->type = CURRENT;
    for (int i = stateId; i < (int)c->ev.size(); i++) c->ev[i] = Ref<StreamEvent>();
    st->nae.push_back(c);
    st->lastScheduled = se->ts + waitingTime;
    sched->notifyAt(st->lastScheduled);
    holder.ret(st);
}
void AbsentPre::resetState() {
    AbsentPreState* st = (AbsentPreState*)holder.get();
    st->pending.clear();
    if (isStart) {
        if (stateType == SH_SEQUENCE && thisPost->nextEveryPre == nullptr &&
            !thisPost->nextPre->pendingList()->empty()) {
            holder.ret(st);
            return;
        }
        init();
    }
    holder.ret(st);
}
// AbsentStreamPreStateProcessor.process(ComplexEventChunk), :150-227
void AbsentPre::processTimer(int64_t currentTime) {
    AbsentPreState* st = (AbsentPreState*)holder.get();
    if (!st->active) {
        holder.ret(st);
        return;
    }
    Chunk<StateEvent> retc;
    bool initialize = isStart && st->nae.empty() && st->pending.empty();
    if (initialize && stateType == SH_SEQUENCE && thisPost->nextEveryPre == nullptr && st->lastScheduled > 0)
        initialize = false;
    if (initialize) {
        SE se = q->newStateEvent();
        addState(se);
    } else if (stateType == SH_SEQUENCE && !st->nae.empty()) {
        resetState();
    }
    updateState();
    for (auto it = st->pending.begin(); it != st->pending.end();) {
        SE ev = *it;
        if (isExpired(ev.get(), currentTime)) {
            it = st->pending.erase(it);
            if (withinEvery && thisPost->nextEveryPre != this) thisPost->nextEveryPre->addEveryState(ev);
            continue;
        }
        if ((ev->ts == -1 && currentTime >= st->lastScheduled) ||
            (ev->ts != -1 && currentTime >= ev->ts + waitingTime)) {
            it = st->pending.erase(it);
            ev->ts = currentTime;
            retc.add(ev);
            continue;
        }
        ++it;
    }
    if (withinEvery) withinEvery->updateState();
    bool notProcessed = !retc.first;
    while (retc.hasNext()) {
        SE se = retc.next();
        retc.remove();
        sendEvent(se, st);
    }
    int64_t actual = q->app->clock;
    if (actual > waitingTime + currentTime) st->lastScheduled = actual + waitingTime;
    if (notProcessed && st->lastScheduled < currentTime) {
        st->lastScheduled = currentTime + waitingTime;
        sched->notifyAt(st->lastScheduled);
    }
    holder.ret(st);
}
void AbsentPre::sendEvent(const SE& se, AbsentPreState* st) {
    if (thisPost->nextProc) {
        Chunk<StateEvent> c(se, se);
        thisPost->nextProc->process(c);
    }
    if (thisPost->nextPre) thisPost->nextPre->addState(se);
    if (thisPost->nextEveryPre)
        thisPost->nextEveryPre->addEveryState(se);
    else if (isStart)
        st->active = false;
    if (thisPost->callbackPre) thisPost->callbackPre->startStateReset();
}
Chunk<StateEvent> AbsentPre::processAndReturn(const Ref<StreamEvent>& sev) {
    AbsentPreState* st = (AbsentPreState*)holder.get();
    if (!st->active) {
        holder.ret(st);
        return Chunk<StateEvent>();
    }
    StreamPre::processAndReturn(sev);
    holder.ret(st);
    return Chunk<StateEvent>();
}
void AbsentPre::partitionCreated() {
    AbsentPreState* st = (AbsentPreState*)holder.get();
    if (!st->started) {
        st->started = true;
        if (isStart && waitingTime != -1 && st->active) {
            st->lastScheduled = q->app->clock + waitingTime;
            sched->notifyAt(st->lastScheduled);
        }
    }
    holder.ret(st);
}
// AbsentStreamPostStateProcessor.java:36-56
void AbsentPost::processSE(const SE& se, Chunk<StateEvent>& c) {
    // the arrival of the absent event kills the partial and re-arms the timer
    thisPre->stateChanged();
    StreamEvent* s = se->ev[stateId].get();
    se->ts = s->ts;
    returned = true;
    if (thisPre->isStart && nextEveryPre && nextEveryPre == thisPre) nextEveryPre->addEveryState(se);
    ((AbsentPre*)thisPre)->updateLastArrivalTime(s->ts);
    (void)c;
}


// ------------------------------------------------------------ AbsentLogical
// AbsentLogicalPreStateProcessor.java:65-420 (event-time semantics)
// StateEvent.addEvent (StateEvent.java:212-222): append to the slot's chain
static void addEventToSlot(StateEvent* se, int slot, const Ref<StreamEvent>& ev) {
    if (!se->ev[slot]) {
        se->ev[slot] = ev;
        return;
    }
    StreamEvent* x = se->ev[slot].get();
    while (x->next) x = x->next.get();
    x->next = ev;
}
// :67-76
void AbsentLogicalPre::updateLastArrivalTime(int64_t ts) {
    LogicalAbsentState* st = (LogicalAbsentState*)holder.get();
    st->lastArrivalTime = ts;
    holder.ret(st);
}
// :78-98
void AbsentLogicalPre::addStateImpl(const SE& se, PreState* pst) {
    LogicalAbsentState* st = (LogicalAbsentState*)pst;
    if (!st->active) return;
    LogicalPre::addStateImpl(se, pst);
    if (!isStart && waitingTime != -1) {
        sched->notifyAt(se->ts + waitingTime);
        if (partner->kind == K_ABSENT_LOGICAL) {
            AbsentLogicalPre* pa = (AbsentLogicalPre*)partner;
            pa->sched->notifyAt(se->ts + pa->waitingTime);
        }
    }
}
// :100-118
void AbsentLogicalPre::addEveryState(const SE& se) {
    SE c = q->copyStateEvent(se);
    c->type = CURRENT;
    if (c->ev[stateId]) c->ts = c->ev[stateId]->ts;  // the last arrived event's timestamp
    c->ev[stateId] = Ref<StreamEvent>();
    c->ev[partner->stateId] = Ref<StreamEvent>();
    PreState* st = holder.get();
    st->nae.push_back(c);
    partner->addToNae(c);
    holder.ret(st);
}
// :120-209
void AbsentLogicalPre::processTimer(int64_t currentTime) {
    LogicalAbsentState* st = (LogicalAbsentState*)holder.get();
    if (!st->active) {
        holder.ret(st);
        return;
    }
    bool notProcessed = true;
    Chunk<StateEvent> retc;
    if (currentTime >= st->lastArrivalTime + waitingTime) {
        if (isStart && stateType == SH_SEQUENCE && st->nae.empty() && st->pending.empty()) {
            SE se = q->newStateEvent();
            addState(se);
        } else if (stateType == SH_SEQUENCE && !st->nae.empty()) {
            resetState();
        }
        updateState();
        SE expired;
        for (auto it = st->pending.begin(); it != st->pending.end();) {
            SE se = *it;
            if (isExpired(se.get(), currentTime)) {  // within
                expired = se;
                it = st->pending.erase(it);
                continue;
            }
            if (waitingTimePassed(currentTime, se.get())) {
                it = st->pending.erase(it);
                const bool partnerIn = (bool)se->ev[partner->stateId];
                if (logicalType == SH_E_LOGICAL_OR && !partnerIn) {
                    // OR: the partner never arrived
                    addEventToSlot(se.get(), stateId, Ref<StreamEvent>(new StreamEvent()));
                    retc.add(se);
                } else if (logicalType == SH_E_LOGICAL_AND && partnerIn) {
                    // AND: the partner arrived but could not send out
                    retc.add(se);
                } else if (logicalType == SH_E_LOGICAL_AND && !partnerIn) {
                    // AND: the partner has not arrived; it may proceed later
                    addEventToSlot(se.get(), stateId, Ref<StreamEvent>(new StreamEvent()));
                }
                continue;
            }
            ++it;
        }
        if (expired && withinEvery) {
            withinEvery->addEveryState(expired);
            withinEvery->updateState();
        }
        retc.reset();
        notProcessed = !retc.first;
        while (retc.hasNext()) {
            SE se = retc.next();
            retc.remove();
            se->ts = currentTime;
            sendEvent(se, st);
        }
        st->lastArrivalTime = 0;
    }
    if (thisPost->nextEveryPre || (notProcessed && isStart)) {
        // every, or an unanswered start state: wait again
        const int64_t nextBreak =
            st->lastArrivalTime == 0 ? q->app->clock + waitingTime : st->lastArrivalTime + waitingTime;
        sched->notifyAt(nextBreak);
    }
    holder.ret(st);
}
// :220-228
bool AbsentLogicalPre::waitingTimePassed(int64_t now, StateEvent* se) {
    if (!se->ev[stateId]) return now >= se->ts + waitingTime;
    return now >= se->ev[stateId]->ts + waitingTime;  // re-added by `every`
}
// :230-251
void AbsentLogicalPre::sendEvent(const SE& se, LogicalAbsentState* st) {
    if (thisPost->nextProc) {
        Chunk<StateEvent> c(se, se);
        thisPost->nextProc->process(c);
    }
    if (thisPost->nextPre) thisPost->nextPre->addState(se);
    if (thisPost->nextEveryPre) {
        thisPost->nextEveryPre->addEveryState(se);
    } else if (isStart) {
        st->active = false;
        if (logicalType == SH_E_LOGICAL_OR && partner->kind == K_ABSENT_LOGICAL)
            ((AbsentLogicalPre*)partner)->setActive(false);
    }
    if (thisPost->callbackPre) thisPost->callbackPre->startStateReset();
}
void AbsentLogicalPre::setActive(bool a) {
    LogicalAbsentState* st = (LogicalAbsentState*)holder.get();
    st->active = a;
    holder.ret(st);
}
// :262-320
Chunk<StateEvent> AbsentLogicalPre::processAndReturn(const Ref<StreamEvent>& sev) {
    Chunk<StateEvent> ret;
    LogicalAbsentState* st = (LogicalAbsentState*)holder.get();
    if (!st->active) {
        holder.ret(st);
        return ret;
    }
    for (auto it = st->pending.begin(); it != st->pending.end();) {
        SE se = *it;
        if (logicalType == SH_E_LOGICAL_OR && se->ev[partner->stateId]) {
            it = st->pending.erase(it);
            continue;
        }
        Ref<StreamEvent> currentStreamEvent = se->ev[stateId];
        se->ev[stateId] = QueryRT::copyStreamEvent(sev);
        processSE(se);
        if (waitingTime != -1 ||
            (stateType == SH_SEQUENCE && logicalType == SH_E_LOGICAL_AND && thisPost->nextEveryPre))
            se->ev[stateId] = currentStreamEvent;  // back to the original state
        bool erased = false;
        if (thisLast->returned) {
            // passed the filter: no longer an absence candidate
            thisLast->returned = false;
            it = st->pending.erase(it);
            erased = true;
            if (stateType == SH_SEQUENCE) partner->pendingList()->remove(se);
        }
        if (!st->changed) {
            se->ev[stateId] = currentStreamEvent;
            if (stateType == SH_SEQUENCE && !erased) {
                it = st->pending.erase(it);
                erased = true;
            }
        }
        if (!erased) ++it;
    }
    holder.ret(st);
    return ret;
}
// :333-351
void AbsentLogicalPre::partitionCreated() {
    LogicalAbsentState* st = (LogicalAbsentState*)holder.get();
    if (!st->started) {
        st->started = true;
        if (isStart && waitingTime != -1 && st->active) sched->notifyAt(q->app->clock + waitingTime);
    }
    holder.ret(st);
}
// :353-388
bool AbsentLogicalPre::partnerCanProceed(StateEvent* se) {
    LogicalAbsentState* st = (LogicalAbsentState*)holder.get();
    bool process;
    if (stateType == SH_SEQUENCE && !thisPost->nextEveryPre && st->lastArrivalTime > 0) {
        process = false;
    } else if (waitingTime == -1) {
        // no `for`: proceed while this absent state has not seen its event
        if (!thisPost->nextEveryPre) {
            process = !se->ev[stateId];
        } else if (st->lastArrivalTime > 0) {
            process = false;
            st->lastArrivalTime = 0;
            init();
        } else {
            process = true;
        }
    } else {
        process = (bool)se->ev[stateId];
    }
    holder.ret(st);
    return process;
}
// AbsentLogicalPostStateProcessor.java:37-49
void AbsentLogicalPost::processSE(const SE& se, Chunk<StateEvent>& c) {
    (void)c;
    thisPre->stateChanged();
    StreamEvent* s = se->ev[stateId].get();
    returned = true;  // tells the pre-processor the absent event arrived
    ((AbsentLogicalPre*)thisPre)->updateLastArrivalTime(s->ts);
}

// Scheduler.java:74-99,171-206 (event-time mode)
void Scheduler::notifyAt(int64_t t) {
    SchedState* st = holder.get();
    st->toNotify.push_back(t);
    holder.ret(st);
}
// sendTimerEvents works on the state object it was handed (no getState)
void Scheduler::sendTimerEvents(SchedState* st, int64_t now) {
    while (!st->toNotify.empty() && st->toNotify.front() <= now) {
        int64_t t = st->toNotify.front();
        st->toNotify.pop_front();
        target(t);
    }
}
int64_t Scheduler::nextDue() const {
    int64_t t = INT64_MAX;
    if (holder.single && !holder.single->toNotify.empty()) t = holder.single->toNotify.front();
    for (auto& kv : holder.states)
        if (!kv.second->toNotify.empty()) t = std::min(t, kv.second->toNotify.front());
    return t;
}
// Scheduler.java:285-300 outside playback: each state's EventCaller runs at its
// head's due time and drains every notify time <= the current time. States due
// at the same instant are independent callers; they run in HashMap order here.
void Scheduler::fireAllDue(int64_t now) {
    std::vector<int64_t> due;
    if (holder.partitioned) {
        order.forEach([&](int64_t k) {
            SchedState* st = holder.states[k];
            if (!st->toNotify.empty() && st->toNotify.front() <= now) due.push_back(k);
        });
    } else {
        SchedState* st = holder.single;
        if (st && !st->toNotify.empty() && st->toNotify.front() <= now) sendTimerEvents(st, now);
        return;
    }
    for (int64_t k : due) {
        auto it = holder.states.find(k);
        if (it == holder.states.end()) continue;
        int64_t saved = app->flow.key;
        if (holder.partitioned) app->flow.key = k;
        sendTimerEvents(it->second, now);
        app->flow.key = saved;
    }
}
void Scheduler::onTimeChange(int64_t now) {
    if (!holder.partitioned) {
        SchedState* st = holder.get();
        bool due = !st->toNotify.empty() && st->toNotify.front() <= now;
        holder.ret(st);
        if (due) sendTimerEvents(st, now);
        return;
    }
    // getAllStates(): every state is in use until returnAllStates
    for (auto& kv : holder.states) kv.second->use++;
    // sortedExpires: TreeMultimap<Long, SchedulerState> with compareTo()==0 for
    // states => the first state in HashMap iteration order per distinct due time
    std::map<int64_t, int64_t> sorted;
    order.forEach([&](int64_t k) {
        SchedState* st = holder.states[k];
        if (!st->toNotify.empty() && st->toNotify.front() <= now) sorted.emplace(st->toNotify.front(), k);
    });
    for (auto& kv : sorted) {
        int64_t saved = app->flow.key;
        app->flow.key = kv.second;
        sendTimerEvents(holder.states[kv.second], now);
        app->flow.key = saved;
    }
    // returnAllStates(): in iteration order, iterator.remove() of every state that
    // canDestroy (HashIterator.remove -> removeNode(..., movable = false))
    for (int64_t k : order.keys()) {
        auto it = holder.states.find(k);
        SchedState* st = it->second;
        st->use--;
        if (st->use == 0 && st->canDestroy()) {
            holder.states.erase(it);
            if (holder.cst == st) holder.cst = nullptr;
            app->zombies.push_back(st);
            order.remove(k, false);
        }
    }
}

// ------------------------------------------------------------ selector
// QuerySelector.java:161-313 + aggregators
// GroupByKeyGenerator.constructEventKey (GroupByKeyGenerator.java:60-71): the group-by
// values' toString() joined by KEY_DELIMITER; equal strings <=> equal (value, null)
// pairs with every NaN of a type alike (Float/Double.toString prints "NaN")
std::vector<int64_t> Selector::groupKey(StateEvent* se) {
    std::vector<int64_t> k;
    for (int i = 0; i < q->d.n_group; i++) {
        Val v = q->eval(q->d.group_expr[i], se);
        int64_t b = v.null ? 0 : v.b;
        if (!v.null && v.t == SH_T_FLOAT && (b & 0x7F800000ll) == 0x7F800000ll && (b & 0x7FFFFFll)) b = 0x7FC00000ll;
        if (!v.null && v.t == SH_T_DOUBLE && std::isnan(asD(v))) b = 0x7FF8000000000000ll;
        k.push_back(b);
        k.push_back(v.null ? 1 : 0);
    }
    return k;
}

void Selector::populate(StateEvent* se) {
    int64_t key = q->app->flow.key;
    AggState* as = nullptr;
    if (containsAggregator) {
        AggState*& a = q->d.n_group > 0 ? aggG[std::make_pair(key, groupKey(se))] : agg[key];
        if (!a) {
            a = new AggState();
            size_t n = q->outs.size();
            a->dsum.assign(n, 0.0);
            a->lsum.assign(n, 0);
            a->cnt.assign(n, 0);
            a->mx.assign(n, Val());
        }
        as = a;
    }
    for (size_t i = 0; i < q->outs.size(); i++) {
        const sh_output_attr& o = q->outs[i];
        if (o.agg == SH_AGG_NONE) {
            Val v = q->eval(o.expr, se);
            v.t = (int8_t)o.type;
            se->out[i] = v;
            continue;
        }
        bool add = se->type == CURRENT;  // EXPIRED -> processRemove
        Val arg = o.expr >= 0 ? q->eval(o.expr, se) : mkBool(true);
        Val r;
        r.t = (int8_t)o.type;
        switch (o.agg) {
            case SH_AGG_SUM: {
                if (arg.null) {
                    // AttributeAggregatorExecutor: null data -> current value
                } else if (arg.t == SH_T_INT || arg.t == SH_T_LONG) {
                    as->lsum[i] += add ? asL(arg) : -asL(arg);
                    as->cnt[i] += add ? 1 : -1;
                } else {
                    as->dsum[i] += add ? asD(arg) : -asD(arg);
                    as->cnt[i] += add ? 1 : -1;
                }
                if (as->cnt[i] == 0 && !add) {
                    r.null = true;
                } else {
                    r.null = false;
                    r.b = o.type == SH_T_LONG ? as->lsum[i] : bf64(as->dsum[i]);
                }
                break;
            }
            case SH_AGG_AVG: {
                if (!arg.null) {
                    as->dsum[i] += add ? asD(arg) : -asD(arg);
                    as->cnt[i] += add ? 1 : -1;
                }
                if (as->cnt[i] == 0) {
                    r.null = true;
                } else {
                    r.null = false;
                    r.b = bf64(as->dsum[i] / (double)as->cnt[i]);
                }
                break;
            }
            case SH_AGG_COUNT: {
                as->cnt[i] += add ? 1 : -1;
                r.null = false;
                r.b = as->cnt[i];
                break;
            }
            case SH_AGG_MAX:
            case SH_AGG_MIN: {
                if (!arg.null && add) {
                    Val& m = as->mx[i];
                    bool better = m.null || (o.agg == SH_AGG_MAX ? cmp(SH_OP_GT, arg, m) : cmp(SH_OP_LT, arg, m));
                    if (better) m = arg;
                }
                r = as->mx[i];
                r.t = (int8_t)o.type;
                break;
            }
        }
        se->out[i] = r;
    }
}
// havingConditionExecutor.execute (a ConditionExpressionExecutor: null is false)
bool Selector::having(StateEvent* se) {
    if (q->d.having < 0) return true;
    const Val v = q->eval(q->d.having, se);
    return !v.null && v.b;
}
// Integer/Long/Float/Double/Boolean.compareTo (OrderByEventComparator.java:73-99);
// Float.compare / Double.compare order by the canonical bits when not < or >
static int javaCompare(const Val& x, const Val& y) {
    switch (x.t) {
        case SH_T_FLOAT: {
            const float a = f32(x.b), b = f32(y.b);
            if (a < b) return -1;
            if (a > b) return 1;
            const int32_t ia = std::isnan(a) ? 0x7fc00000 : (int32_t)(uint32_t)bf32(a);
            const int32_t ib = std::isnan(b) ? 0x7fc00000 : (int32_t)(uint32_t)bf32(b);
            return ia == ib ? 0 : (ia < ib ? -1 : 1);
        }
        case SH_T_DOUBLE: {
            const double a = f64(x.b), b = f64(y.b);
            if (a < b) return -1;
            if (a > b) return 1;
            const int64_t ia = std::isnan(a) ? 0x7ff8000000000000ll : bf64(a);
            const int64_t ib = std::isnan(b) ? 0x7ff8000000000000ll : bf64(b);
            return ia == ib ? 0 : (ia < ib ? -1 : 1);
        }
        case SH_T_BOOL: return (int)(x.b != 0) - (int)(y.b != 0);
        case SH_T_INT: {
            const int32_t a = (int32_t)x.b, b = (int32_t)y.b;
            return a < b ? -1 : (a > b ? 1 : 0);
        }
        default: return x.b < y.b ? -1 : (x.b > y.b ? 1 : 0);
    }
}
// OrderByEventComparator.compare, OrderByEventComparator.java:62-116
int Selector::orderCompare(StateEvent* a, StateEvent* b) {
    for (int i = 0; i < q->d.n_order; i++) {
        const Val x = q->eval(q->d.order_expr[i], a);
        const Val y = q->eval(q->d.order_expr[i], b);
        if (!x.null && !y.null) {
            int r = javaCompare(x, y);
            if ((q->d.order_desc >> i) & 1) r = -r;
            if (r != 0) return r;
        } else if (!x.null) {
            return -1;
        } else if (!y.null) {
            return 1;
        }
    }
    return 0;
}
// QuerySelector.orderEventChunk, QuerySelector.java:452-483
void Selector::orderChunk(Chunk<StateEvent>& c) {
    Chunk<StateEvent> ordering;
    std::vector<SE> list;
    auto flush = [&]() {
        std::stable_sort(list.begin(), list.end(),
                         [&](const SE& a, const SE& b) { return orderCompare(a.get(), b.get()) < 0; });
        for (auto& e : list) ordering.add(e);
        list.clear();
    };
    c.reset();
    if (!c.first) return;
    EvType cur = c.first->type;
    while (c.hasNext()) {
        SE ev = c.next();
        c.remove();
        if (ev->type != cur) {
            cur = ev->type;
            flush();
        }
        list.push_back(ev);
    }
    flush();
    c.clear();
    c.add(ordering.first);
}
// QuerySelector.offsetEventChunk, QuerySelector.java:502-519 (insert into: currentOn only)
void Selector::offsetChunk(Chunk<StateEvent>& c) {
    c.reset();
    int64_t n = 0;
    while (c.hasNext()) {
        SE ev = c.next();
        if (ev->type == CURRENT || ev->type == EXPIRED) {
            if (q->d.offset > n) {
                if (ev->type == CURRENT) n++;
                c.remove();
            } else {
                break;
            }
        }
    }
}
// QuerySelector.limitEventChunk, QuerySelector.java:485-500
void Selector::limitChunk(Chunk<StateEvent>& c) {
    c.reset();
    int64_t n = 0;
    while (c.hasNext()) {
        SE ev = c.next();
        if (ev->type == CURRENT || ev->type == EXPIRED) {
            if (q->d.limit > n && ev->type == CURRENT)
                n++;
            else
                c.remove();
        }
    }
}
// the query's OutputRateLimiter.process: PassThroughOutputRateLimiter,
// FirstPerEventOutputRateLimiter.process (FirstPerEventOutputRateLimiter.java:47-72) or
// LastPerEventOutputRateLimiter.process (LastPerEventOutputRateLimiter.java:45-68), each
// with its counter in a per-partition state (int arithmetic: FIRST with N == 1 never resets)
void Selector::rateProcess(Chunk<StateEvent>& c) {
    const int kind = q->d.rate_kind;
    if (kind == SH_RATE_FIRST_TIME) {
        // FirstPerTimeOutputRateLimiter.process (FirstPerTimeOutputRateLimiter.java:53-75): the
        // chunk's first event passes when the partition's outputTime is null or
        // outputTime + value <= the timestamp generator's current time (playback: the
        // clock InputHandler.send moved), which becomes the new outputTime
        const int64_t now = q->app->clock;
        auto it = rateOutTime.find(q->app->flow.key);
        if (it == rateOutTime.end() || (int64_t)((uint64_t)it->second + (uint64_t)q->d.rate_value) <= now) {
            rateOutTime[q->app->flow.key] = now;
            c.reset();
            SE ev = c.next();
            c.remove();
            Chunk<StateEvent> out;
            out.add(ev);
            out.reset();
            sendToCallBacks(out);
        }
        return;
    }
    if (kind != SH_RATE_FIRST_EVENTS && kind != SH_RATE_LAST_EVENTS && kind != SH_RATE_ALL_EVENTS) {
        sendToCallBacks(c);
        return;
    }
    Chunk<StateEvent> out;
    int32_t& counter = rateCounter[q->app->flow.key];
    c.reset();
    while (c.hasNext()) {
        SE ev = c.next();
        if (kind == SH_RATE_ALL_EVENTS) {
            // AllPerEventOutputRateLimiter.process (AllPerEventOutputRateLimiter.java:48-75): every
            // current / expired event is held; the N-th releases the held chunk
            if (ev->type == CURRENT || ev->type == EXPIRED) {
                c.remove();
                Chunk<StateEvent>& held = rateHeld[q->app->flow.key];
                held.add(ev);
                counter = (int32_t)((uint32_t)counter + 1u);
                if (counter == q->d.rate_value) {
                    out.add(held.first);
                    held.clear();
                    counter = 0;
                }
            }
        } else if (kind == SH_RATE_FIRST_EVENTS) {
            c.remove();
            counter = (int32_t)((uint32_t)counter + 1u);
            if (counter == 1) {
                out.add(ev);
            } else if (counter == q->d.rate_value) {
                counter = 0;
            }
        } else if (ev->type == CURRENT || ev->type == EXPIRED) {
            counter = (int32_t)((uint32_t)counter + 1u);
            if (counter == q->d.rate_value) {
                c.remove();
                out.add(ev);
                counter = 0;
            }
        }
    }
    out.reset();
    if (out.hasNext()) sendToCallBacks(out);
}
void Selector::process(Chunk<StateEvent>& c) {
    if (containsAggregator) {
        // processInBatchNoGroupBy, QuerySelector.java:271-313: the last event that
        // passes `having` is the chunk's output
        c.reset();
        SE lastEv;
        while (c.hasNext()) {
            SE ev = c.next();
            if (ev->type == CURRENT || ev->type == EXPIRED) {
                populate(ev.get());
                ev->sel_seq = q->app->curSeq;
                if (having(ev.get()) && ev->type == CURRENT) {
                    c.remove();
                    lastEv = ev;
                }
            }
        }
        if (lastEv) {
            c.clear();
            c.add(lastEv);
            rateProcess(c);
        }
        return;
    }
    // processNoGroupBy, QuerySelector.java:161-205
    c.reset();
    while (c.hasNext()) {
        SE ev = c.next();
        switch (ev->type) {
            case CURRENT:
            case EXPIRED:
                populate(ev.get());
                ev->sel_seq = q->app->curSeq;
                // currentOn only (insert into); events failing `having` leave the chunk
                if (ev->type != CURRENT || !having(ev.get())) c.remove();
                break;
            case TIMER:
                c.remove();
                break;
            default:
                break;
        }
    }
    if (q->d.n_order > 0) orderChunk(c);
    if (q->d.offset >= 0) offsetChunk(c);
    if (q->d.limit >= 0) limitChunk(c);
    c.reset();
    if (c.hasNext()) rateProcess(c);
}
// OutputRateLimiter.sendToCallBacks, OutputRateLimiter.java:63-106
void Selector::sendToCallBacks(Chunk<StateEvent>& c) {
    App* a = q->app;
    if (a->holder) {
        ReturnHolder* h = a->holder;
        h->chunk.add(c.first);
        h->has = true;
        h->sel = this;
        return;
    }
    if (!c.first) return;
    c.reset();
    while (c.hasNext()) {
        SE ev = c.next();
        if (ev->type == EXPIRED) {
            ev->type = CURRENT;
        } else if (ev->type == RESET) {
            c.remove();
        }
    }
    if (!c.first) return;
    int32_t group = a->cbGroup++;
    for (StateEvent* ev = c.first.get(); ev; ev = ev->next.get()) {
        OutRow r;
        r.query = q->index;
        r.seq = ev->sel_seq;
        r.ts = ev->ts;
        r.v = ev->out;
        r.group = group;
        a->out.push_back(std::move(r));
    }
}

// ------------------------------------------------------------ receivers
void Receiver::setNext(StreamPre* p) {
    if (multi) {
        for (auto& np : nextProcessors)
            if (!np) {
                np = p;
                break;
            }
        // StateMultiProcessStreamReceiver.setNext: querySelector of THIS state's post
        querySelector = dynamic_cast<Selector*>(p->thisPost->nextProc);
    } else {
        nextProcessors[0] = p;
        // SingleProcessStreamReceiver.setNext: querySelector of the last processor
        querySelector = dynamic_cast<Selector*>(p->thisLast->nextProc);
    }
}
void Receiver::stabilizeStates(int64_t ts) {
    for (StreamPre* p : q->pres) p->expireEvents(ts);
    if (q->d.state_type == SH_SEQUENCE) {
        q->root->reset();
        q->root->update();
    } else if (multi) {
        for (StreamPre* p : forStream) p->updateState();
    } else if (!forStream.empty()) {
        forStream[0]->updateState();
    }
}
static Ref<StreamEvent> convert(const Ref<Row>& r) {
    Ref<StreamEvent> s(new StreamEvent());
    s->row = r;
    s->ts = r->ts;
    return s;
}
void Receiver::receive(const std::vector<Ref<Row>>& rows) {
    App* a = q->app;
    if (!multi) {
        // SingleProcessStreamReceiver.processAndClear, :48-73
        Chunk<StateEvent> retc;
        StreamPre* next = nextProcessors[0];
        std::vector<uint64_t> retSeq;
        for (const auto& r : rows) {
            a->curSeq = r->seq;
            stabilizeStates(r->ts);
            Ref<StreamEvent> sev = convert(r);
            Chunk<StateEvent> ec = next->processAndReturn(sev);
            if (ec.first) {
                for (StateEvent* e = ec.first.get(); e; e = e->next.get()) e->sel_seq = r->seq;
                retc.add(ec.first);
            }
            a->flushZombies();
        }
        while (retc.hasNext()) {
            SE se = retc.next();
            retc.remove();
            uint64_t s = se->sel_seq;
            a->curSeq = s;
            Chunk<StateEvent> one(se, se);
            querySelector->process(one);
        }
        a->flushZombies();
        return;
    }
    // MultiProcessStreamReceiver.receive(Event[]), :155-183
    std::vector<std::unique_ptr<ReturnHolder>> list;
    for (const auto& r : rows) {
        a->curSeq = r->seq;
        std::unique_ptr<ReturnHolder> h(new ReturnHolder());
        a->holder = h.get();
        stabilizeStates(r->ts);
        for (int slot : eventSequence) {
            Ref<StreamEvent> ne = convert(r);
            // StateMultiProcessStreamReceiver.processAndClear, :47-68
            Chunk<StateEvent> retc;
            Chunk<StateEvent> ec = nextProcessors[slot]->processAndReturn(ne);
            if (ec.first) retc.add(ec.first);
            ec.clear();
            if (querySelector) {
                while (retc.hasNext()) {
                    SE se = retc.next();
                    retc.remove();
                    Chunk<StateEvent> one(se, se);
                    querySelector->process(one);
                }
            }
            if (a->holder && a->holder->has) {
                list.push_back(std::move(h));
                h.reset(new ReturnHolder());
                a->holder = h.get();
            }
        }
        a->holder = nullptr;
        a->flushZombies();
    }
    for (auto& h : list) {
        if (h->sel) h->sel->sendToCallBacks(h->chunk);
    }
    a->flushZombies();
}

// ------------------------------------------------------------ parse
// StateInputStreamParser.parse, StateInputStreamParser.java:148-408
Inner* QueryRT::parse(int ei, StreamPre* pre, StreamPost* post, std::vector<StreamPre*>& list, bool isStart) {
    const sh_state_elem& e = elems[ei];
    int st = d.state_type;
    switch (e.kind) {
        case SH_E_STREAM:
        case SH_E_ABSENT_STREAM: {
            Receiver* rcv = receivers[e.stream].get();
            int stateIndex = slotCounter++;
            if (stateIndex != e.slot) {
                err = "slot mismatch between descriptor and parse order";
                return nullptr;
            }
            if (!pre) {
                if (e.kind == SH_E_ABSENT_STREAM) {
                    AbsentPre* ap = own<AbsentPre>(e.waiting_ms);
                    startupPres.push_back(ap);
                    Scheduler* s = new Scheduler();
                    scheds.emplace_back(s);
                    s->app = app;
                    s->target = [ap](int64_t t) { ap->processTimer(t); };
                    s->holder.app = app;
                    s->holder.partitioned = partition >= 0;
                    s->holder.factory = []() { return new SchedState(); };
                    if (partition >= 0) {
                        s->holder.order = &s->order;
                        App* ap = app;
                        s->order.string_hash = [ap](int64_t k) { return ap->keyHash(k); };
                        s->order.compare = [ap](int64_t a, int64_t b) { return ap->keyCompare(a, b); };
                    }
                    app->schedulers.push_back(s);
                    ap->sched = s;
                    pre = ap;
                } else {
                    pre = own<StreamPre>();
                }
                pre->q = this;
                pre->stateType = st;
            }
            pre->stateId = stateIndex;
            pre->isStart = isStart;
            // processor chain: pre -> [filter] -> post
            Proc* chain = nullptr;
            if (e.filter >= 0) chain = own<FilterProc>(this, e.filter);
            pre->nextProc = chain;
            if (!post) {
                if (e.kind == SH_E_ABSENT_STREAM)
                    post = own<AbsentPost>();
                else
                    post = own<StreamPost>();
            }
            post->stateId = stateIndex;
            pre->setToLast(post);
            post->thisPre = pre;
            pre->thisPost = post;
            pre->thisLast = post;
            Inner* in = ownI<Inner>();
            in->first = pre;
            in->last = post;
            in->ssr.push_back({rcv, pre});
            list.push_back(pre);
            return in;
        }
        case SH_E_NEXT: {
            Inner* cur = parse(e.child0, pre, post, list, isStart);
            if (!cur) return nullptr;
            Inner* nxt = parse(e.child1, pre, post, list, false);
            if (!nxt) return nullptr;
            cur->last->setNextStatePre(nxt->first);
            NextInner* ni = ownI<NextInner>(cur, nxt);
            ni->first = cur->first;
            ni->last = nxt->last;
            ni->ssr = cur->ssr;
            ni->ssr.insert(ni->ssr.end(), nxt->ssr.begin(), nxt->ssr.end());
            return ni;
        }
        case SH_E_EVERY: {
            std::vector<StreamPre*> wl;
            Inner* in = parse(e.child0, pre, post, wl, isStart);
            if (!in) return nullptr;
            EveryInner* ev = ownI<EveryInner>(in);
            ev->first = in->first;
            ev->last = in->last;
            ev->ssr = in->ssr;
            ev->last->setNextEveryStatePre(ev->first);
            for (StreamPre* p : wl) p->withinEvery = ev->first;
            list.insert(list.end(), wl.begin(), wl.end());
            return ev;
        }
        case SH_E_LOGICAL_AND:
        case SH_E_LOGICAL_OR: {
            int lt = e.kind;
            const sh_state_elem& e1 = elems[e.child0];
            const sh_state_elem& e2 = elems[e.child1];
            // an absent element gets AbsentLogicalPre/Post + its own scheduler
            // (StateInputStreamParser.java:289-344); element 1's scheduler first
            auto make = [&](const sh_state_elem& x) -> LogicalPre* {
                if (x.kind != SH_E_ABSENT_STREAM) return own<LogicalPre>(lt);
                AbsentLogicalPre* ap = own<AbsentLogicalPre>(lt, x.waiting_ms);
                startupPres.push_back(ap);
                Scheduler* s = new Scheduler();
                scheds.emplace_back(s);
                s->app = app;
                s->target = [ap](int64_t t) { ap->processTimer(t); };
                s->holder.app = app;
                s->holder.partitioned = partition >= 0;
                s->holder.factory = []() { return new SchedState(); };
                if (partition >= 0) {
                    s->holder.order = &s->order;
                    App* a2 = app;
                    s->order.string_hash = [a2](int64_t k) { return a2->keyHash(k); };
                    s->order.compare = [a2](int64_t a, int64_t b) { return a2->keyCompare(a, b); };
                }
                app->schedulers.push_back(s);
                ap->sched = s;
                return ap;
            };
            LogicalPre* p1 = make(e1);
            p1->q = this;
            p1->stateType = st;
            LogicalPost* o1 = e1.kind == SH_E_ABSENT_STREAM ? own<AbsentLogicalPost>(lt) : own<LogicalPost>(lt);
            LogicalPre* p2 = make(e2);
            p2->q = this;
            p2->stateType = st;
            LogicalPost* o2 = e2.kind == SH_E_ABSENT_STREAM ? own<AbsentLogicalPost>(lt) : own<LogicalPost>(lt);
            o1->partnerPre = p2;
            o2->partnerPre = p1;
            o1->partnerPost = o2;
            o2->partnerPost = o1;
            p1->partner = p2;
            p2->partner = p1;
            Inner* in2 = parse(e.child1, p2, o2, list, isStart);
            if (!in2) return nullptr;
            Inner* in1 = parse(e.child0, p1, o1, list, isStart);
            if (!in1) return nullptr;
            LogicalInner* li = ownI<LogicalInner>(in1, in2);
            li->first = in1->first;
            li->last = in2->last;
            li->ssr = in2->ssr;
            li->ssr.insert(li->ssr.end(), in1->ssr.begin(), in1->ssr.end());
            return li;
        }
        case SH_E_COUNT: {
            int mn = e.min_count == SH_ANY ? 0 : e.min_count;
            int mx = e.max_count == SH_ANY ? INT32_MAX : e.max_count;
            CountPre* cp = own<CountPre>(mn, mx);
            cp->q = this;
            cp->stateType = st;
            CountPost* co = own<CountPost>(mn, mx);
            cp->countPost = co;
            Inner* in = parse(e.child0, cp, co, list, isStart);
            if (!in) return nullptr;
            Inner* ci = ownI<Inner>();  // CountInnerStateRuntime: same first/last/ssr
            ci->first = in->first;
            ci->last = in->last;
            ci->ssr = in->ssr;
            return ci;
        }
    }
    err = "unknown state element";
    return nullptr;
}

bool QueryRT::build() {
    // receivers: one per stream id, Single if used once, Multi(k) otherwise
    // (StateInputStreamParser.java:91-110)
    std::map<int, int> uses;
    for (auto& e : elems)
        if (e.kind == SH_E_STREAM || e.kind == SH_E_ABSENT_STREAM) uses[e.stream]++;
    for (auto& kv : uses) {
        Receiver* r = new Receiver();
        r->q = this;
        r->stream = kv.first;
        r->processCount = kv.second;
        r->multi = kv.second > 1;
        r->nextProcessors.assign(kv.second, nullptr);
        if (r->multi) {
            for (int i = kv.second - 1; i >= 0; i--) r->eventSequence.push_back(i);
        }
        receivers[kv.first].reset(r);
    }
    for (auto& e : elems)
        if (e.kind == SH_E_STREAM || e.kind == SH_E_ABSENT_STREAM) nslots++;
    selector = own<Selector>();
    selector->q = this;
    for (auto& o : outs)
        if (o.agg != SH_AGG_NONE) selector->containsAggregator = true;
    root = parse(d.root, nullptr, nullptr, pres, true);
    if (!root) return false;
    for (StreamPre* p : pres) {
        p->holder.app = app;
        p->holder.partitioned = partition >= 0;
        StreamPre* pp = p;
        p->holder.factory = [pp]() { return pp->newState(); };
    }
    if (d.within_ms >= 0) {
        std::vector<int> ids;
        for (StreamPre* p : pres)
            if (p->isStart) ids.push_back(p->stateId);
        for (StreamPre* p : pres) {
            p->startIds = ids;
            p->within = d.within_ms;
        }
    }
    root->first->thisLast = root->last;
    // StateStreamRuntime.setCommonProcessor: setQuerySelector then setup
    root->setQuerySelector(selector);
    root->setup();
    return true;
}

// StateStreamRuntime.initPartition, StateStreamRuntime.java:90-97
void QueryRT::initPartition() {
    root->init();
    for (StreamPre* p : startupPres) {
        if (p->kind == K_ABSENT) ((AbsentPre*)p)->partitionCreated();
        if (p->kind == K_ABSENT_LOGICAL) ((AbsentLogicalPre*)p)->partitionCreated();
    }
}

}  // namespace ref

using namespace ref;

struct ref_app {
    App a;
};

extern "C" {

ref_app* ref_create(const sh_app_desc* d, char* err, int errlen) {
    auto fail = [&](const std::string& m) -> ref_app* {
        if (err && errlen > 0) snprintf(err, errlen, "%s", m.c_str());
        return nullptr;
    };
    if (!d || d->version != SH_DESC_VERSION) return fail("bad descriptor version");
    ref_app* ra = new ref_app();
    App& a = ra->a;
    a.d = *d;
    for (int s = 0; s < d->n_streams; s++)
        a.streamTypes.emplace_back(d->streams[s].attr_types, d->streams[s].attr_types + d->streams[s].n_attrs);
    a.partitions.resize(d->n_partitions);
    if (d->n_partitions) a.partStreams.assign(d->partition_streams, d->partition_streams + d->n_partitions * d->n_streams);
    a.subs.resize(d->n_streams);
    std::set<std::pair<int, int>> partSub;
    for (int qi = 0; qi < d->n_queries; qi++) {
        const sh_query_desc& qd = d->queries[qi];
        QueryRT* q = new QueryRT();
        a.queries.emplace_back(q);
        q->app = &a;
        q->index = qi;
        q->d = qd;
        q->elems.assign(qd.elems, qd.elems + qd.n_elems);
        q->exprs.assign(qd.exprs, qd.exprs + qd.n_exprs);
        q->outs.assign(qd.outputs, qd.outputs + qd.n_outputs);
        q->partition = qd.partition;
        if (!q->build()) {
            std::string m = q->err;
            delete ra;
            return fail("query " + std::to_string(qi) + ": " + m);
        }
        std::string serr;
        if (qd.n_order < 0 || qd.n_order > SH_MAX_ORDER) serr = "order by: 0..4 attributes";
        for (int i = 0; i < qd.n_order && serr.empty(); i++) {
            const int e = qd.order_expr[i];
            if (e < 0 || e >= qd.n_exprs)
                serr = "order by: expression out of range";
            else if (qd.exprs[e].type == SH_T_STRING || qd.exprs[e].type == SH_T_OBJECT)
                serr = "order by: string / object attributes are outside the restatement";
        }
        bool agg = false;
        for (int o = 0; o < qd.n_outputs; o++) agg |= qd.outputs[o].agg != SH_AGG_NONE;
        // processInBatchNoGroupBy would pass an empty chunk on (QuerySelector.java:304-311)
        if (agg && (qd.offset > 0 || qd.limit == 0)) serr = "aggregating selector with offset > 0 or limit 0";
        if (qd.rate_kind != SH_RATE_NONE &&
            ((qd.rate_kind != SH_RATE_FIRST_EVENTS && qd.rate_kind != SH_RATE_LAST_EVENTS &&
              qd.rate_kind != SH_RATE_ALL_EVENTS && qd.rate_kind != SH_RATE_FIRST_TIME) ||
             qd.rate_value < (qd.rate_kind == SH_RATE_FIRST_TIME ? 0 : 1)))
            serr = "output rate limiting: `output [first|last|all] every N events` or `output first every T`";
        if (qd.rate_kind == SH_RATE_FIRST_TIME && !d->playback)
            serr = "output first every T: the limiter reads the wall clock outside @app:playback";
        if (!serr.empty()) {
            delete ra;
            return fail("query " + std::to_string(qi) + ": " + serr);
        }
        if (qd.partition >= 0) a.partitions[qd.partition].queries.push_back(q);
        for (auto& kv : q->receivers) {
            int s = kv.first;
            if (qd.partition >= 0) {
                if (!partSub.count({s, qd.partition})) {
                    partSub.insert({s, qd.partition});
                    a.subs[s].push_back(-1 - qd.partition);
                }
            } else {
                a.subs[s].push_back(qi);
            }
        }
    }
    return ra;
}

void ref_start(ref_app* ra) {
    App& a = ra->a;
    for (auto& q : a.queries)
        if (q->partition < 0) q->initPartition();
    a.flushZombies();
}

int ref_send(ref_app* ra, const sh_batch* b, uint64_t first_seq) {
    App& a = ra->a;
    if (!b || b->on_device || b->stream < 0 || b->stream >= a.d.n_streams) return SH_E_INVALID_ARG;
    int s = b->stream;
    const auto& types = a.streamTypes[s];
    std::vector<Ref<Row>> rows;
    rows.reserve(b->n);
    for (int64_t i = 0; i < b->n; i++) {
        Row* r = new Row();
        r->ts = b->ts[i];
        r->seq = first_seq + i;
        r->stream = s;
        r->v.resize(types.size());
        r->nul.assign(types.size(), 0);
        for (size_t c = 0; c < types.size(); c++) {
            const void* col = b->cols[c];
            switch (types[c]) {
                case SH_T_LONG: r->v[c] = ((const int64_t*)col)[i]; break;
                case SH_T_FLOAT: r->v[c] = bf32(((const float*)col)[i]); break;
                case SH_T_DOUBLE: r->v[c] = bf64(((const double*)col)[i]); break;
                case SH_T_BOOL: r->v[c] = ((const uint8_t*)col)[i] ? 1 : 0; break;
                default: r->v[c] = ((const int32_t*)col)[i]; break;
            }
            if (b->nulls && b->nulls[c]) r->nul[c] = b->nulls[c][i];
        }
        rows.emplace_back(r);
    }
    if (rows.empty()) return SH_OK;
    // InputHandler.send: playback clock moves to the batch's last timestamp and
    // fires due timers BEFORE the batch (InputHandler.java:85-96); rows a timer
    // emits carry the batch's first sequence number as their trigger
    a.nextSeq = first_seq;
    if (a.d.playback) ref_advance_time(ra, rows.back()->ts);
    a.nextSeq = first_seq + (uint64_t)rows.size();
    for (int sub : a.subs[s]) {
        if (sub >= 0) {
            QueryRT* q = a.queries[sub].get();
            a.flow.key = INT64_MIN;
            q->receivers[s]->receive(rows);
        } else {
            int p = -1 - sub;
            PartitionRT& pr = a.partitions[p];
            // PartitionStreamReceiver.receive(Event[]): consecutive same-key runs
            size_t i = 0;
            while (i < rows.size()) {
                int32_t key = b->keys ? b->keys[i] : 0;
                size_t j = i + 1;
                if (key < 0) {  // null key: event dropped
                    i = j;
                    continue;
                }
                while (j < rows.size() && (b->keys ? b->keys[j] : 0) == key) j++;
                std::vector<Ref<Row>> run(rows.begin() + i, rows.begin() + j);
                a.flow.key = key;
                if (!pr.seen.count(key)) {
                    for (QueryRT* q : pr.queries) q->initPartition();
                    pr.seen.insert(key);
                }
                for (QueryRT* q : pr.queries) {
                    auto it = q->receivers.find(s);
                    if (it != q->receivers.end()) it->second->receive(run);
                }
                a.flow.key = INT64_MIN;
                a.flushZombies();
                i = j;
            }
        }
    }
    a.flow.key = INT64_MIN;
    a.flushZombies();
    return SH_OK;
}

int ref_set_partition_keys(ref_app* ra, int32_t first, int32_t n, const uint16_t* utf16, const int64_t* offsets) {
    if (!ra || first < 0 || n < 0 || (n && (!utf16 || !offsets))) return SH_E_INVALID_ARG;
    App& a = ra->a;
    const size_t need = (size_t)first + (size_t)n;
    if (a.keyStr.size() < need) {
        a.keyStr.resize(need);
        a.keyHas.resize(need, 0);
        a.keyHashes.resize(need, 0);
    }
    for (int32_t i = 0; i < n; i++) {
        a.keyStr[first + i].assign((const char16_t*)utf16 + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
        a.keyHas[first + i] = 1;
        a.keyHashes[first + i] = java_string_hash(utf16 + offsets[i], offsets[i + 1] - offsets[i]);
    }
    return SH_OK;
}

int ref_advance_time(ref_app* ra, int64_t now) {
    App& a = ra->a;
    if (now < a.clock) return SH_OK;  // TimestampGeneratorImpl: time never goes back
    a.curSeq = a.nextSeq;
    if (!a.d.playback) {
        // wall clock: the clock passes through every queued notify time in
        // order and each due state fires at exactly its due time
        for (;;) {
            int64_t t = INT64_MAX;
            for (Scheduler* s : a.schedulers) t = std::min(t, s->nextDue());
            if (t > now) break;
            a.clock = std::max(a.clock, t);
            for (Scheduler* s : a.schedulers) s->fireAllDue(a.clock);
            a.flow.key = INT64_MIN;
        }
        a.clock = now;
        a.flushZombies();
        return SH_OK;
    }
    a.clock = now;
    for (Scheduler* s : a.schedulers) s->onTimeChange(now);
    a.flow.key = INT64_MIN;
    a.flushZombies();
    return SH_OK;
}

int64_t ref_out_count(ref_app* ra) { return (int64_t)ra->a.out.size(); }

int ref_out_read(ref_app* ra, int64_t start, int64_t count, int32_t* query, uint64_t* seq, int64_t* ts,
                 int64_t* values, uint8_t* nulls, int32_t n_out, int32_t* cb_group) {
    App& a = ra->a;
    if (start < 0 || start + count > (int64_t)a.out.size()) return SH_E_INVALID_ARG;
    for (int64_t i = 0; i < count; i++) {
        const OutRow& r = a.out[start + i];
        if (query) query[i] = r.query;
        if (seq) seq[i] = r.seq;
        if (ts) ts[i] = r.ts;
        if (cb_group) cb_group[i] = r.group;
        for (int c = 0; c < n_out; c++) {
            bool has = c < (int)r.v.size();
            if (values) values[i * n_out + c] = has ? r.v[c].b : 0;
            if (nulls) nulls[i * n_out + c] = has ? (uint8_t)r.v[c].null : 1;
        }
    }
    return SH_OK;
}

void ref_out_clear(ref_app* ra) { ra->a.out.clear(); }

int64_t ref_list_get(ref_app* ra, int64_t list, int64_t cap, int64_t* values, uint8_t* nulls) {
    App& a = ra->a;
    if (list < 0 || list >= (int64_t)a.listV.size()) return -1;
    const auto& v = a.listV[list];
    const auto& nl = a.listN[list];
    for (int64_t i = 0; i < (int64_t)v.size() && i < cap; i++) {
        if (values) values[i] = v[i];
        if (nulls) nulls[i] = nl[i];
    }
    return (int64_t)v.size();
}

void ref_destroy(ref_app* ra) { delete ra; }

const char* ref_last_error(ref_app* ra) { return ra->a.err.c_str(); }

}  // extern "C"
