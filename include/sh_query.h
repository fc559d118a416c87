/*
 * sh_query.h — the lowered pattern/sequence app descriptor that crosses the
 * drop-in boundary.
 *
 * This is the flat, C-ABI image of what siddhi-core's query compiler hands to
 * StateInputStreamParser: the StateElement tree of each pattern/sequence query
 * (query-api `io.siddhi.query.api.execution.query.input.state.*`), its filter
 * expressions, its selector and the `partition with (attr of Stream)` spec.
 *
 *   reference: modules/siddhi-core/src/main/java/io/siddhi/core/util/parser/
 *              StateInputStreamParser.java:76-408   (element tree -> processors)
 *              ExpressionParser.java:225-1439        (typed expression executors)
 *              SelectorParser.java:215               (select-clause executors)
 *              core/partition/PartitionStreamReceiver.java:176-272 (value partitions)
 *
 * Nothing in here is a torch type: plain structs, pointers and sizes. The same
 * descriptor feeds the product (libsiddhi_hip.so, sh_compile) and the CPU
 * oracle (oracle/librefcpu.so, tests only).
 *
 * Values: every attribute / constant value travels as 8 raw bytes (int64_t):
 *   SH_T_INT    int32 sign-extended          SH_T_LONG   int64
 *   SH_T_FLOAT  IEEE-754 binary32 bits (low) SH_T_DOUBLE IEEE-754 binary64 bits
 *   SH_T_BOOL   0 / 1                        SH_T_STRING host dictionary id (int32)
 * String equality is dictionary-id equality (the host owns one dictionary per
 * app runtime), which is exactly String.equals for the compare executors
 * (EqualCompareConditionExpressionExecutorStringString.java:34).
 */
#ifndef SH_QUERY_H
#define SH_QUERY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SH_DESC_VERSION 5
#define SH_MAX_ORDER 4
#define SH_MAX_GROUP 4

/* Attribute.Type (api/definition/Attribute.java) */
enum sh_type {
    SH_T_STRING = 0,
    SH_T_INT = 1,
    SH_T_LONG = 2,
    SH_T_FLOAT = 3,
    SH_T_DOUBLE = 4,
    SH_T_BOOL = 5,
    SH_T_OBJECT = 6
};

/* StateInputStream.Type */
enum sh_state_type { SH_PATTERN = 0, SH_SEQUENCE = 1 };

/* StateElement kinds (api/execution/query/input/state/) */
enum sh_elem_kind {
    SH_E_STREAM = 0,        /* StreamStateElement            */
    SH_E_ABSENT_STREAM = 1, /* AbsentStreamStateElement      */
    SH_E_NEXT = 2,          /* NextStateElement  (a -> b, a, b) */
    SH_E_EVERY = 3,         /* EveryStateElement             */
    SH_E_LOGICAL_AND = 4,   /* LogicalStateElement AND       */
    SH_E_LOGICAL_OR = 5,    /* LogicalStateElement OR        */
    SH_E_COUNT = 6          /* CountStateElement <m:n> + * ? */
};

/* Expression operators (core/executor/..) */
enum sh_op {
    SH_OP_CONST = 0,   /* ConstantExpressionExecutor                     */
    SH_OP_VAR = 1,     /* VariableExpressionExecutor (state slot, chain index, attr) */
    SH_OP_AND = 2,     /* AndConditionExpressionExecutor                 */
    SH_OP_OR = 3,      /* OrConditionExpressionExecutor                  */
    SH_OP_NOT = 4,     /* NotConditionExpressionExecutor                 */
    SH_OP_EQ = 5,      /* compare/equal/..                                */
    SH_OP_NE = 6,      /* compare/notequal/..                             */
    SH_OP_GT = 7,      /* compare/greaterthan/..                          */
    SH_OP_GE = 8,      /* compare/greaterthanequal/..                     */
    SH_OP_LT = 9,      /* compare/lessthan/..                             */
    SH_OP_LE = 10,     /* compare/lessthanequal/..                        */
    SH_OP_ADD = 11,    /* math/add/..                                     */
    SH_OP_SUB = 12,    /* math/subtract/..                                */
    SH_OP_MUL = 13,    /* math/multiply/..                                */
    SH_OP_DIV = 14,    /* math/divide/..                                  */
    SH_OP_MOD = 15,    /* math/mod/..                                     */
    SH_OP_IS_NULL = 16,        /* IsNullConditionExpressionExecutor      */
    SH_OP_IS_NULL_STREAM = 17, /* IsNullStreamConditionExpressionExecutor (e1 is null) */
    SH_OP_IF_THEN_ELSE = 18,   /* function/IfThenElseFunctionExecutor (cond=lhs, a=rhs, b=third) */
    SH_OP_BOOL_VAR = 19,       /* BoolConditionExpressionExecutor wrapping a BOOL expr */
    SH_OP_OUTPUT = 20,         /* having: output attribute `attr` of the selected event
                                  (HAVING_STATE variables, ExpressionParser.java:1308-1318) */
    SH_OP_MULTI_VAR = 21       /* select of a count state's attribute without an index:
                                  MultiValueVariableFunctionExecutor (core/executor/
                                  MultiValueVariableFunctionExecutor.java:39-70, chosen at
                                  ExpressionParser.java:1385-1437) -- attribute `attr` of every
                                  event of slot `slot`'s chain from index `chain` on, as a List;
                                  type OBJECT, ltype = the attribute's type. Output rows carry
                                  a list handle (sh_list_get). */
};

/* select-clause aggregators (query/selector/attribute/aggregator/) */
enum sh_agg { SH_AGG_NONE = 0, SH_AGG_SUM = 1, SH_AGG_AVG = 2, SH_AGG_COUNT = 3,
              SH_AGG_MAX = 4, SH_AGG_MIN = 5 };

/* chain-index sentinels, SiddhiConstants.java:90-91 */
#define SH_CHAIN_CURRENT (-1) /* last event of the slot's chain            */
#define SH_CHAIN_LAST (-2)    /* second-to-last event of the slot's chain  */
/* <= -3 : (chain length + index)-th element, StateEvent.java:166-179 */

#define SH_ANY (-1)           /* CountStateElement.ANY */

typedef struct sh_expr {
    int32_t op;        /* enum sh_op                                       */
    int32_t type;      /* result type (enum sh_type)                       */
    int32_t lhs;       /* operand expr index or -1                         */
    int32_t rhs;       /* operand expr index or -1                         */
    int32_t third;     /* IF_THEN_ELSE else-branch, else -1                */
    int32_t ltype;     /* operand types: select the typed executor         */
    int32_t rtype;
    int32_t slot;      /* VAR / IS_NULL_STREAM: stream-event chain index (state slot) */
    int32_t chain;     /* VAR: index in the slot's event chain (>=0, CURRENT, LAST, <=-3) */
    int32_t attr;      /* VAR: attribute position in the stream definition */
    int32_t is_null;   /* CONST: the constant is null                      */
    int32_t pad;
    int64_t cval;      /* CONST: raw 8-byte value                          */
} sh_expr;

typedef struct sh_state_elem {
    int32_t kind;      /* enum sh_elem_kind                                */
    int32_t child0;    /* NEXT: current; EVERY/COUNT: inner; LOGICAL: element 1 */
    int32_t child1;    /* NEXT: next; LOGICAL: element 2                   */
    int32_t stream;    /* STREAM/ABSENT_STREAM: stream index in the app    */
    int32_t filter;    /* STREAM/ABSENT_STREAM: filter expr root, or -1    */
    int32_t slot;      /* STREAM/ABSENT_STREAM: state slot = MetaStateEvent position
                          assigned in StateInputStreamParser parse order   */
    int32_t min_count; /* COUNT: min (SH_ANY)                               */
    int32_t max_count; /* COUNT: max (SH_ANY)                               */
    int64_t waiting_ms;/* ABSENT_STREAM: `for` time in ms                   */
} sh_state_elem;

typedef struct sh_output_attr {
    int32_t expr;      /* expression root (aggregator argument when agg != NONE; -1 for count()) */
    int32_t agg;       /* enum sh_agg                                       */
    int32_t type;      /* output attribute type                             */
    int32_t pad;
} sh_output_attr;

typedef struct sh_stream_def {
    int32_t n_attrs;
    int32_t pad;
    const int32_t* attr_types;   /* n_attrs entries of enum sh_type          */
} sh_stream_def;

typedef struct sh_query_desc {
    int32_t state_type;          /* enum sh_state_type                       */
    int32_t root;                /* root element index                       */
    int32_t n_elems;
    int32_t n_exprs;
    int32_t n_outputs;
    int32_t n_slots;             /* number of stream state elements (MetaStateEvent size) */
    int32_t partition;           /* index of the enclosing partition, -1 if none */
    int32_t output_stream;       /* app-level output stream id (insert into)   */
    int64_t within_ms;           /* `within` in ms, -1 if absent               */
    const sh_state_elem* elems;
    const sh_expr* exprs;
    const sh_output_attr* outputs;
    int32_t having;              /* having condition root (QuerySelector havingConditionExecutor,
                                    SelectorParser.java:248-260), -1 if none */
    int32_t n_order;             /* `order by` attributes (OrderByEventComparator, SelectorParser.java:110-114), 0 if none */
    int32_t order_expr[SH_MAX_ORDER]; /* variable expression per order-by attribute (HAVING_STATE resolution);
                                    INT / LONG / FLOAT / DOUBLE / BOOL (string order needs the text) */
    int32_t order_desc;          /* bit i: attribute i is DESC                  */
    int32_t rate_kind;           /* enum sh_rate: the query's OutputRateLimiter (OutputParser.constructOutputRateLimiter) */
    int64_t limit;               /* QuerySelector.limit, -1 if none (SelectorParser.java:115-123) */
    int64_t offset;              /* QuerySelector.offset, -1 if none (:124-132)  */
    int32_t rate_value;          /* events per period (SH_RATE_FIRST_EVENTS / _LAST_EVENTS / _ALL_EVENTS),
                                    or the period in ms (SH_RATE_FIRST_TIME) */
    int32_t n_group;             /* `group by` attributes (GroupByKeyGenerator, SelectorParser.java:102-108), 0 if none */
    int32_t group_expr[SH_MAX_GROUP]; /* variable expression per group-by attribute (UNKNOWN_STATE, default index 0):
                                    the aggregators keep one state per (partition key, group key) */
} sh_query_desc;

/* output rate limiting (query/output/ratelimit/): PassThroughOutputRateLimiter,
   `output first every N events` (FirstPerEventOutputRateLimiter.java:47-72) or
   `output last every N events` (LastPerEventOutputRateLimiter.java:45-68) */
enum sh_rate { SH_RATE_NONE = 0, SH_RATE_FIRST_EVENTS = 1, SH_RATE_LAST_EVENTS = 2,
               SH_RATE_ALL_EVENTS = 3, /* `output [all] every N events`: AllPerEventOutputRateLimiter */
               SH_RATE_FIRST_TIME = 4  /* `output first every T` (rate_value = T in ms), playback apps:
                                          FirstPerTimeOutputRateLimiter.java:53-75 against the playback clock */ };

typedef struct sh_app_desc {
    int32_t version;             /* SH_DESC_VERSION                            */
    int32_t n_streams;
    int32_t n_queries;
    int32_t n_partitions;
    int32_t playback;            /* @app:playback                              */
    int32_t pad;
    const sh_stream_def* streams;
    const sh_query_desc* queries;/* in app (junction subscription) order     */
    /* partition p is keyed, per stream, by the host-computed key ids passed with
       each batch (ValuePartitionExecutor: key = attr.toString()); a stream
       participates in partition p iff partition_streams[p*n_streams+s] != 0 */
    const uint8_t* partition_streams;
    /* partition_attr[p*n_streams+s]: attribute index of stream s that keys
       partition p (`partition with (attr of Stream)`), -1 if not keyed or
       range-partitioned (keys computed by the host from the ranges) */
    const int32_t* partition_attr;
} sh_app_desc;

#ifdef __cplusplus
}
#endif
#endif /* SH_QUERY_H */
