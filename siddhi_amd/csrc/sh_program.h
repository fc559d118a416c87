// sh_program.h — the device NFA table ("program") that sh_compile lowers a
// pattern query to, shared by the host lowering (sh_host.cpp) and the gfx950
// kernels (sh_kernels.hip).
//
// Lowering follows StateInputStreamParser.parseInputStream/parse
// (core/util/parser/StateInputStreamParser.java:76-408) for the class of
// queries the device engine runs: PATTERN chains of stream states
// (`[every] e0=S0[f0] -> e1=S1[f1] -> ... [within T]`), optionally
// partitioned. Filters and select expressions become typed postfix bytecode
// with the reference executors' conversion and null rules
// (core/executor/condition/**, core/executor/math/**).
#pragma once
#include <stdint.h>

#define SHP_MAX_STATES 8
#define SHP_MAX_OUT 16
#define SHP_MAX_CODE 512
#define SHP_MAX_STACK 16
#define SHP_MAX_STREAMS 8

// compare / arithmetic domains (Java binary numeric promotion of the operands)
enum shp_dom { DOM_I32 = 0, DOM_I64 = 1, DOM_F32 = 2, DOM_F64 = 3, DOM_STR = 4, DOM_BOOL = 5 };

enum shp_opcode {
    OPC_CONST = 0,      // x = const index
    OPC_VAR = 1,        // a = slot, b = attr, c = type, x = chain index
    OPC_AND = 2,
    OPC_OR = 3,
    OPC_NOT = 4,
    OPC_BOOLV = 5,
    OPC_CMP = 6,        // a = sh_op (EQ..LE), b = domain
    OPC_ARITH = 7,      // a = sh_op (ADD..MOD), b = result type
    OPC_ISNULL = 8,
    OPC_ISNULL_STREAM = 9,  // a = slot, x = chain index
    OPC_SELECT = 10,    // if-then-else: pops else, then, cond
    OPC_CAST = 11,      // b = target type (retag only)
    OPC_OUTPUT = 12     // having: b = output attribute, c = its type
};

struct shp_instr {
    uint8_t op, a, b, c;
    int32_t x;
};

// A conjunct `lhs op rhs` of a filter that needs no stack machine:
// lhs is an attribute, rhs an attribute, a constant, or `attribute (aop) constant`.
struct shp_term {
    uint8_t op;     // SH_OP_EQ..SH_OP_LE
    uint8_t dom;    // compare domain (enum shp_dom)
    uint8_t lslot, lattr, ltype;
    uint8_t rkind;  // 0: attribute, 1: constant, 2: attribute (aop) constant
    uint8_t rslot, rattr, rtype;
    uint8_t aop;    // SH_OP_ADD/SUB/MUL for rkind 2
    uint8_t atype;  // arithmetic result type for rkind 2
    uint8_t ctype;  // constant type
    int64_t c;      // constant raw bits
};

#define SHP_MAX_TERMS 4

struct shp_program {
    int32_t n_states;                 // chain length
    int32_t every_start;              // `every` wraps exactly the start state
    int32_t window_ok;                // shape runs on the window engine (sh_window.hip)
    int64_t within_ms;                // -1: none
    int32_t n_streams;
    int32_t n_out;
    int32_t state_stream[SHP_MAX_STATES];
    int32_t filter_pc[SHP_MAX_STATES];   // -1: no filter
    int32_t filter_len[SHP_MAX_STATES];
    // register-only form of the filters: conjunction of shp_term (no nulls)
    int32_t filter_fast[SHP_MAX_STATES];
    int32_t filter_nterms[SHP_MAX_STATES];
    shp_term terms[SHP_MAX_STATES][SHP_MAX_TERMS];
    // projection-only select: output o reads attribute (out_slot, out_attr)
    int32_t out_fast;
    int32_t out_slot[SHP_MAX_OUT];
    int32_t out_attr[SHP_MAX_OUT];
    // aggregators (sum / avg / count of a plain attribute) on the fast engines:
    // (out_slot, out_attr) is the argument, turned into the running value per
    // partition key by the post-pass over the ordered rows (sh_agg.hip)
    int32_t agg_post;
    // per stream: which states update (stabilizeStates) and the processing order
    // (eventSequence: reverse of setup order), PatternSingle/MultiProcessStreamReceiver
    int32_t upd_count[SHP_MAX_STREAMS];
    int32_t upd_state[SHP_MAX_STREAMS][SHP_MAX_STATES];
    int32_t proc_count[SHP_MAX_STREAMS];
    int32_t proc_state[SHP_MAX_STREAMS][SHP_MAX_STATES];
    int32_t out_pc[SHP_MAX_OUT];
    int32_t out_len[SHP_MAX_OUT];
    int32_t out_agg[SHP_MAX_OUT];        // enum sh_agg
    int32_t out_type[SHP_MAX_OUT];       // enum sh_type
    int32_t out_arg_type[SHP_MAX_OUT];   // aggregator argument type
    int32_t stream_nattr[SHP_MAX_STREAMS];
    int32_t attr_type[SHP_MAX_STREAMS][32];
    int32_t n_code;
    int32_t n_const;
    shp_instr code[SHP_MAX_CODE];
    int64_t consts[64];
    uint8_t const_null[64];
    uint8_t const_type[64];
};

// per-key state record layout (bytes), computed on the host
struct shp_layout {
    int32_t cap;            // partial capacity per list
    int32_t rec_words;      // 8-byte words per partial record: ts + ceil(n_states*4/8)
    int64_t key_bytes;      // stride between keys
    int64_t off_lists;      // offset of state 1's pending list
    int64_t list_bytes;     // bytes per list (cap * rec_words * 8)
    int64_t off_agg;        // aggregator block offset
};
