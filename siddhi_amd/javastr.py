"""Java's toString() of partition-key values and the UTF-16 packing the C-ABI
takes them in (sh_set_partition_keys).

ValuePartitionExecutor keys a partition by ``attr.toString()``
(core/partition/executor/ValuePartitionExecutor.java:34-40); the playback
scheduler's state map hashes those Strings (String.hashCode), so the host must
hand the library the exact Java text:
  String          itself
  Integer / Long  decimal
  Boolean         "true" / "false"
  Float / Double  Float.toString / Double.toString: plain decimal for
                  1e-3 <= |x| < 1e7, else d.dddE[-]n; shortest round-trip digits
                  (OpenJDK's FloatingDecimal matches the shortest form except for
                  rare values it prints with one digit more -- parity unpinned
                  for float / double partition keys)
"""
from __future__ import annotations

import math

import numpy as np


def _java_fp(digits: str, exp10: int, neg: bool) -> str:
    """digits: significant digits d1d2...dk (no leading zeros), value = 0.d1...dk x 10^exp10"""
    sign = "-" if neg else ""
    k = len(digits)
    e = exp10 - 1  # scientific exponent of d1.d2...
    if -3 <= e < 7:
        if e >= 0:
            ip = digits[: e + 1].ljust(e + 1, "0")
            fp = digits[e + 1:] or "0"
        else:
            ip = "0"
            fp = "0" * (-e - 1) + digits
        return f"{sign}{ip}.{fp}"
    mant = digits[0] + "." + (digits[1:] or "0")
    return f"{sign}{mant}E{e}"


def _split_repr(r: str):
    """shortest repr text (Python / numpy) -> (digits, exp10) with value = 0.digits x 10^exp10"""
    r = r.lstrip("-")
    if "e" in r or "E" in r:
        m, ex = r.lower().split("e")
        ex = int(ex)
    else:
        m, ex = r, 0
    if "." in m:
        ip, fp = m.split(".")
    else:
        ip, fp = m, ""
    digits = (ip + fp).lstrip("0")
    lead = len(ip) - (len(ip + fp) - len((ip + fp).lstrip("0")))
    exp10 = ex + lead
    digits = digits.rstrip("0") or "0"
    return digits, exp10


def java_double_to_string(x: float) -> str:
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    d, e = _split_repr(repr(abs(x)))
    return _java_fp(d, e, x < 0)


def java_float_to_string(x) -> str:
    f = np.float32(x)
    if np.isnan(f):
        return "NaN"
    if np.isinf(f):
        return "Infinity" if f > 0 else "-Infinity"
    if f == 0:
        return "-0.0" if np.signbit(f) else "0.0"
    r = np.format_float_scientific(np.abs(f), unique=True, trim="-")
    d, e = _split_repr(r)
    return _java_fp(d, e, bool(np.signbit(f)))


def java_string_hash(s: str) -> int:
    """String.hashCode (UTF-16 code units, 32-bit wrap-around, signed)"""
    h = 0
    for cu in np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16):
        h = (31 * h + int(cu)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def pack_utf16(strings):
    """list of str -> (uint16 code units, int64 offsets[n + 1])"""
    parts = [np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16) for s in strings]
    offs = np.zeros(len(parts) + 1, dtype=np.int64)
    if parts:
        offs[1:] = np.cumsum([len(p) for p in parts])
        chars = np.concatenate(parts) if offs[-1] else np.zeros(1, np.uint16)
    else:
        chars = np.zeros(1, np.uint16)
    return np.ascontiguousarray(chars), offs


def dense_key_strings(prefix: str, n: int, width: int = 8):
    """UTF-16 of prefix + zero-padded decimal id for ids 0..n-1, vectorised:
    (uint16 code units, int64 offsets[n + 1])"""
    pre = np.frombuffer(prefix.encode("utf-16-le"), dtype=np.uint16)
    L = len(pre) + width
    ids = np.arange(n, dtype=np.int64)
    out = np.empty((n, L), dtype=np.uint16)
    out[:, : len(pre)] = pre
    for i in range(width):
        out[:, len(pre) + width - 1 - i] = ord("0") + (ids // 10 ** i) % 10
    offs = np.arange(n + 1, dtype=np.int64) * L
    return out.reshape(-1), offs
