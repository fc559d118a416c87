"""ctypes mirror of include/sh_query.h and include/siddhi_hip.h (the C-ABI boundary)."""
import ctypes as C

SH_DESC_VERSION = 5
SH_MAX_ORDER = 4
SH_MAX_GROUP = 4

SH_OK = 0
SH_E_INVALID_ARG = -1
SH_E_OOM = -2
SH_E_HIP = -3
SH_E_UNSUPPORTED = -4
SH_E_STATE_OVERFLOW = -5
SH_E_MORE = -6
SH_E_NO_DEVICE = -7

STATUS_NAMES = {0: "OK", -1: "INVALID_ARG", -2: "OOM", -3: "HIP", -4: "UNSUPPORTED",
                -5: "STATE_OVERFLOW", -6: "MORE", -7: "NO_DEVICE"}


class sh_expr(C.Structure):
    _fields_ = [("op", C.c_int32), ("type", C.c_int32), ("lhs", C.c_int32), ("rhs", C.c_int32),
                ("third", C.c_int32), ("ltype", C.c_int32), ("rtype", C.c_int32),
                ("slot", C.c_int32), ("chain", C.c_int32), ("attr", C.c_int32),
                ("is_null", C.c_int32), ("pad", C.c_int32), ("cval", C.c_int64)]


class sh_state_elem(C.Structure):
    _fields_ = [("kind", C.c_int32), ("child0", C.c_int32), ("child1", C.c_int32),
                ("stream", C.c_int32), ("filter", C.c_int32), ("slot", C.c_int32),
                ("min_count", C.c_int32), ("max_count", C.c_int32), ("waiting_ms", C.c_int64)]


class sh_output_attr(C.Structure):
    _fields_ = [("expr", C.c_int32), ("agg", C.c_int32), ("type", C.c_int32), ("pad", C.c_int32)]


class sh_stream_def(C.Structure):
    _fields_ = [("n_attrs", C.c_int32), ("pad", C.c_int32), ("attr_types", C.POINTER(C.c_int32))]


class sh_query_desc(C.Structure):
    _fields_ = [("state_type", C.c_int32), ("root", C.c_int32), ("n_elems", C.c_int32),
                ("n_exprs", C.c_int32), ("n_outputs", C.c_int32), ("n_slots", C.c_int32),
                ("partition", C.c_int32), ("output_stream", C.c_int32), ("within_ms", C.c_int64),
                ("elems", C.POINTER(sh_state_elem)), ("exprs", C.POINTER(sh_expr)),
                ("outputs", C.POINTER(sh_output_attr)), ("having", C.c_int32), ("n_order", C.c_int32),
                ("order_expr", C.c_int32 * SH_MAX_ORDER), ("order_desc", C.c_int32), ("rate_kind", C.c_int32),
                ("limit", C.c_int64), ("offset", C.c_int64), ("rate_value", C.c_int32), ("n_group", C.c_int32),
                ("group_expr", C.c_int32 * SH_MAX_GROUP)]


class sh_app_desc(C.Structure):
    _fields_ = [("version", C.c_int32), ("n_streams", C.c_int32), ("n_queries", C.c_int32),
                ("n_partitions", C.c_int32), ("playback", C.c_int32), ("pad", C.c_int32),
                ("streams", C.POINTER(sh_stream_def)), ("queries", C.POINTER(sh_query_desc)),
                ("partition_streams", C.POINTER(C.c_uint8)),
                ("partition_attr", C.POINTER(C.c_int32))]


class sh_batch(C.Structure):
    _fields_ = [("stream", C.c_int32), ("on_device", C.c_int32), ("n", C.c_int64),
                ("ts", C.c_void_p), ("keys", C.c_void_p),
                ("cols", C.POINTER(C.c_void_p)), ("nulls", C.POINTER(C.c_void_p))]


class sh_match_buf(C.Structure):
    _fields_ = [("capacity", C.c_int64), ("count", C.c_int64),
                ("query", C.POINTER(C.c_int32)), ("trigger_seq", C.POINTER(C.c_uint64)),
                ("ts", C.POINTER(C.c_int64)), ("values", C.POINTER(C.c_int64)),
                ("nulls", C.POINTER(C.c_uint8)), ("n_out", C.c_int32), ("pad", C.c_int32)]


class sh_device_run(C.Structure):
    _fields_ = [("n", C.c_int64), ("d_ts", C.c_void_p), ("d_keys", C.c_void_p),
                ("n_keys", C.c_int32), ("batch_events", C.c_int32), ("d_cols", C.POINTER(C.c_void_p)),
                ("out_capacity", C.c_int64), ("d_out_seq", C.c_void_p),
                ("d_out_values", C.c_void_p), ("out_count", C.c_int64), ("stream", C.c_void_p),
                ("d_out_query", C.c_void_p), ("d_out_cols", C.POINTER(C.c_void_p)),
                # end of the V1 struct (SH_DEVICE_RUN_V1_BYTES); read by sh_run_device_v2 only
                ("version", C.c_int32), ("out_layout", C.c_int32), ("d_run", C.c_void_p)]


SH_DEVICE_RUN_V2 = 2
SH_OUT_RAW = 0
SH_OUT_PACKED = 1


class sh_due_cand(C.Structure):
    _fields_ = [("t", C.c_int64), ("order", C.c_uint64), ("key", C.c_int32), ("pad", C.c_int32)]


# sh_coordinator callbacks (include/siddhi_hip.h, key-sharded streaming)
HISTORY_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_int64,
                         C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.c_int64))
SELECT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int32, C.POINTER(sh_due_cand), C.c_int64,
                        C.POINTER(C.c_int64), C.POINTER(C.c_int64))
MIN_TIME_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64, C.POINTER(C.c_int64))


class sh_coordinator(C.Structure):
    _fields_ = [("user", C.c_void_p), ("history", HISTORY_FN), ("select", SELECT_FN), ("min_time", MIN_TIME_FN)]


class sh_kernel_times(C.Structure):
    _fields_ = [("segment_ms", C.c_float), ("advance_ms", C.c_float), ("emit_ms", C.c_float),
                ("total_ms", C.c_float), ("advance_launches", C.c_int64)]


# every symbol include/siddhi_hip.h declares (checked by tests/test_abi.py)
EXPORTED = ["sh_start", "sh_compile", "sh_push_batch", "sh_advance_time", "sh_drain", "sh_pending",
            "sh_destroy", "sh_last_error", "sh_run_device", "sh_run_device_v2", "sh_last_kernel_times",
            "sh_version", "sh_device_count", "sh_set_partition_keys", "sh_snapshot", "sh_restore",
            "sh_set_coordinator", "sh_push_batch_part", "sh_drain_ordered", "sh_list_get",
            "sh_packed_row_layout"]


def bind_product(lib):
    lib.sh_compile.argtypes = [C.POINTER(sh_app_desc), C.POINTER(C.c_void_p)]
    lib.sh_compile.restype = C.c_int
    lib.sh_start.argtypes = [C.c_void_p]
    lib.sh_start.restype = C.c_int
    lib.sh_push_batch.argtypes = [C.c_void_p, C.POINTER(sh_batch)]
    lib.sh_push_batch.restype = C.c_int
    lib.sh_advance_time.argtypes = [C.c_void_p, C.c_int64]
    lib.sh_advance_time.restype = C.c_int
    lib.sh_drain.argtypes = [C.c_void_p, C.POINTER(sh_match_buf)]
    lib.sh_drain.restype = C.c_int
    lib.sh_pending.argtypes = [C.c_void_p]
    lib.sh_pending.restype = C.c_int64
    lib.sh_destroy.argtypes = [C.c_void_p]
    lib.sh_destroy.restype = None
    lib.sh_last_error.argtypes = [C.c_void_p]
    lib.sh_last_error.restype = C.c_char_p
    lib.sh_set_partition_keys.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
    lib.sh_set_partition_keys.restype = C.c_int
    lib.sh_run_device.argtypes = [C.c_void_p, C.POINTER(sh_device_run)]
    lib.sh_run_device.restype = C.c_int
    lib.sh_run_device_v2.argtypes = [C.c_void_p, C.POINTER(sh_device_run)]
    lib.sh_run_device_v2.restype = C.c_int
    lib.sh_last_kernel_times.argtypes = [C.c_void_p, C.POINTER(sh_kernel_times)]
    lib.sh_last_kernel_times.restype = C.c_int
    lib.sh_packed_row_layout.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.c_int32, C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int32)]
    lib.sh_packed_row_layout.restype = C.c_int
    lib.sh_snapshot.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
    lib.sh_snapshot.restype = C.c_int
    lib.sh_restore.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    lib.sh_restore.restype = C.c_int
    lib.sh_set_coordinator.argtypes = [C.c_void_p, C.POINTER(sh_coordinator)]
    lib.sh_set_coordinator.restype = C.c_int
    lib.sh_push_batch_part.argtypes = [C.c_void_p, C.POINTER(sh_batch), C.c_void_p, C.c_int64, C.c_int64]
    lib.sh_push_batch_part.restype = C.c_int
    lib.sh_drain_ordered.argtypes = [C.c_void_p, C.POINTER(sh_match_buf), C.c_void_p]
    lib.sh_drain_ordered.restype = C.c_int
    lib.sh_list_get.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]
    lib.sh_list_get.restype = C.c_int64
    lib.sh_version.argtypes = []
    lib.sh_version.restype = C.c_char_p
    lib.sh_device_count.argtypes = []
    lib.sh_device_count.restype = C.c_int
    # diagnostics of the hipRTC window kernels (not part of the reference-facing ABI)
    lib.shx_jit_status.argtypes = [C.c_void_p]
    lib.shx_jit_status.restype = C.c_int
    lib.shx_jit_compile.argtypes = [C.c_void_p]
    lib.shx_jit_compile.restype = C.c_int
    lib.shx_jit_source.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
    lib.shx_jit_source.restype = C.c_int64
    lib.shx_bucket_compile.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
    lib.shx_bucket_compile.restype = C.c_int
    lib.shx_bucket_status.argtypes = [C.c_void_p]
    lib.shx_bucket_status.restype = C.c_int
    lib.shx_seq3_status.argtypes = [C.c_void_p]
    lib.shx_seq3_status.restype = C.c_int
    lib.shx_agg_status.argtypes = [C.c_void_p]
    lib.shx_agg_status.restype = C.c_int
    lib.shx_rules_status.argtypes = [C.c_void_p]
    lib.shx_rules_status.restype = C.c_int
    lib.shx_host_profile.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    lib.shx_host_profile.restype = C.c_int
    lib.shx_seq3_shape.argtypes = [C.c_void_p]
    lib.shx_seq3_shape.restype = C.c_int
    return lib


def bind_oracle(lib):
    lib.ref_create.argtypes = [C.POINTER(sh_app_desc), C.c_char_p, C.c_int]
    lib.ref_create.restype = C.c_void_p
    lib.ref_start.argtypes = [C.c_void_p]
    lib.ref_start.restype = None
    lib.ref_send.argtypes = [C.c_void_p, C.POINTER(sh_batch), C.c_uint64]
    lib.ref_send.restype = C.c_int
    lib.ref_set_partition_keys.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
    lib.ref_set_partition_keys.restype = C.c_int
    lib.ref_advance_time.argtypes = [C.c_void_p, C.c_int64]
    lib.ref_advance_time.restype = C.c_int
    lib.ref_out_count.argtypes = [C.c_void_p]
    lib.ref_out_count.restype = C.c_int64
    lib.ref_out_read.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    lib.ref_out_read.restype = C.c_int
    lib.ref_out_clear.argtypes = [C.c_void_p]
    lib.ref_out_clear.restype = None
    lib.ref_list_get.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]
    lib.ref_list_get.restype = C.c_int64
    lib.ref_destroy.argtypes = [C.c_void_p]
    lib.ref_destroy.restype = None
    return lib


def object_columns(compiled):
    """per query, the select positions of type OBJECT (List values of
    SH_OP_MULTI_VAR outputs, MultiValueVariableFunctionExecutor)"""
    return [[k for k, t in enumerate(q.out_types) if t == 6] for q in compiled.queries]


def resolve_lists(out, obj_cols, get):
    """out: a drain dict; obj_cols: object_columns(compiled); get(handle) ->
    (values int64[], nulls uint8[]) while the handles are valid. Adds
    out["lists"] = {(row, col): (values, nulls)} for every List value."""
    import numpy as np
    lists = {}
    if any(obj_cols):
        q = out["query"]
        for r in range(len(q)):
            cols = obj_cols[int(q[r])] if 0 <= int(q[r]) < len(obj_cols) else []
            for c in cols:
                if not out["nulls"][r, c]:
                    v, nl = get(int(out["values"][r, c]))
                    lists[(r, c)] = (np.asarray(v, np.int64), np.asarray(nl, np.uint8))
    out["lists"] = lists
    return out


def list_getter(fn, h):
    """get(handle) over a C function fn(h, handle, cap, values, nulls) -> length"""
    import numpy as np

    def get(handle):
        n = int(fn(h, handle, 0, None, None))
        if n < 0:
            raise RuntimeError(f"no list {handle}")
        v = np.zeros(max(n, 1), np.int64)
        nl = np.zeros(max(n, 1), np.uint8)
        fn(h, handle, n, v.ctypes.data, nl.ctypes.data)
        return v[:n], nl[:n]
    return get


def concat_drains(parts):
    """drain dicts of consecutive drains as one (List values re-keyed by row)"""
    import numpy as np
    keys = [k for k in parts[-1] if k != "lists"]
    out = {k: np.concatenate([p[k] for p in parts]) for k in keys}
    lists, base = {}, 0
    for p in parts:
        for (r, c), v in (p.get("lists") or {}).items():
            lists[(r + base, c)] = v
        base += len(p["query"])
    out["lists"] = lists
    return out
