"""ctypes mirror of include/tsdbhip.h (the C-ABI of libtsdbhip.so).

Only plain pointers and sizes cross the boundary; this module holds the
struct layouts and constants shared by the host adapter (opentsdb_amd.core)
and the test harness.
"""
import ctypes as C

ABI_VERSION = 7
PATH_ALIGNED_GROUP = 1  # tsdbhip_timing.paths (include/tsdbhip.h)
PATH_ALIGNED_RERUN = 2
PATH_LOCKSTEP = 4  # k_lockstep: one pass over the qualifiers and values of a lockstep group
PATH_DIRECT_REDO = 8  # its proposal did not hold: the call ran again on the proven path
PATH_UNIFORM = 16  # every kept span proposed one class key at assembly: G from the key, one round trip
PATH_UNIFORM_FALLBACK = 32  # the uniform aligned group did not stand: the general path ran the call

OK = 0
E_ILLEGAL_DATA = -1
E_NAN_INF = -2
E_EMPTY_SPAN = -3
E_CAPACITY = -4
E_HIP = -5
E_RCCL = -6
E_INVALID_ARG = -7
E_UNSORTED = -8
E_OUT_OF_BOUNDS = -9
E_NO_DEVICE = -10
E_UNSUPPORTED = -11

ERR_NAMES = {
    OK: "OK", E_ILLEGAL_DATA: "E_ILLEGAL_DATA", E_NAN_INF: "E_NAN_INF",
    E_EMPTY_SPAN: "E_EMPTY_SPAN", E_CAPACITY: "E_CAPACITY", E_HIP: "E_HIP",
    E_RCCL: "E_RCCL", E_INVALID_ARG: "E_INVALID_ARG", E_UNSORTED: "E_UNSORTED",
    E_OUT_OF_BOUNDS: "E_OUT_OF_BOUNDS", E_NO_DEVICE: "E_NO_DEVICE",
}

AGG_SUM, AGG_MIN, AGG_MAX, AGG_AVG, AGG_DEV = 0, 1, 2, 3, 4

DESC_DEVICE = 0x1
EXACT_ORDER = 0x2
SHARDED = 0x4

ROW_NONE, ROW_SINGLE, ROW_TRIVIAL, ROW_COMPLEX, ROW_ERROR, ROW_OOB = 0, 1, 2, 3, 4, 5

SYN_INT64_COUNTER, SYN_FLOAT32, SYN_FLOAT64 = 0, 1, 2

UNIQUE_ID_BYTES = 128

P8 = C.POINTER(C.c_uint8)
P16 = C.POINTER(C.c_uint16)
P32 = C.POINTER(C.c_uint32)
P64 = C.POINTER(C.c_uint64)
PI64 = C.POINTER(C.c_int64)


class SgDesc(C.Structure):
    _fields_ = [
        ("start_time", C.c_int64),
        ("end_time", C.c_int64),
        ("rate", C.c_uint8),
        ("agg", C.c_uint8),
        ("ds_agg", C.c_uint8),
        ("reserved0", C.c_uint8),
        ("flags", C.c_uint32),
        ("ds_interval", C.c_int32),
        ("n_spans", C.c_uint32),
        ("n_rows", C.c_uint64),
        ("span_row_start", P64),
        ("row_base", P32),
        ("row_ncells", P32),
        ("row_qual_off", P64),
        ("row_val_off", P64),
        ("row_val_len", P32),
        ("qual_bytes", P8),
        ("qual_nbytes", C.c_uint64),
        ("val_bytes", P8),
        ("val_nbytes", C.c_uint64),
        ("span0", C.c_uint64),
    ]


class SgOut(C.Structure):
    _fields_ = [
        ("capacity", C.c_uint64),
        ("ts", PI64),
        ("is_int", P8),
        ("bits", PI64),
        ("n_out", C.c_uint64),
        ("n_input_points", C.c_uint64),
        ("err_code", C.c_int32),
        ("reserved0", C.c_int32),
        ("err_index", C.c_int64),
    ]


HOT_NONE, HOT_DS_CHUNKS, HOT_DECODE_FAST, HOT_DECODE_GEN = 0, 1, 2, 3
HOT_NAMES = {1: "k_ds_reg+k_ds_spans", 2: "k_decode_fast", 3: "k_decode_general", 4: "k_compact_wave",
             5: "k_reduce", 6: "k_lockstep", 7: "k_ug_ds_reg", 8: "k_ug_dev", 9: "k_ds_reg"}


class Timing(C.Structure):
    _fields_ = [
        ("total_ms", C.c_float),
        ("decode_ms", C.c_float),
        ("grid_ms", C.c_float),
        ("reduce_ms", C.c_float),
        ("exchange_ms", C.c_float),
        ("hot_ms", C.c_float),
        ("hot_kernel", C.c_uint32),
        ("n_collectives", C.c_uint32),
        ("decode_bytes", C.c_uint64),
        ("alg_bytes", C.c_uint64),
        ("n_grid", C.c_uint64),
        ("n_emitted", C.c_uint64),
        ("paths", C.c_uint32),
        ("late_stamp", C.c_uint32),
        ("x_bytes", C.c_uint64),
        ("h2d_bytes", C.c_uint64),
    ]


class RowsDesc(C.Structure):
    _fields_ = [
        ("flags", C.c_uint32),
        ("reserved0", C.c_uint32),
        ("n_rows", C.c_uint64),
        ("n_kvs", C.c_uint64),
        ("row_kv_start", P64),
        ("row_qual_off", P64),
        ("row_val_off", P64),
        ("kv_qual_len", P16),
        ("kv_val_len", P16),
        ("qual_bytes", P8),
        ("qual_nbytes", C.c_uint64),
        ("val_bytes", P8),
        ("val_nbytes", C.c_uint64),
    ]


class RowsOut(C.Structure):
    _fields_ = [
        ("qual_capacity", C.c_uint64),
        ("val_capacity", C.c_uint64),
        ("row_status", P8),
        ("row_qual_off", P64),
        ("row_qual_len", P32),
        ("row_val_off", P64),
        ("row_val_len", P32),
        ("qual_bytes", P8),
        ("val_bytes", P8),
        ("qual_used", C.c_uint64),
        ("val_used", C.c_uint64),
        ("n_complex", C.c_uint64),
        ("row_write", P8),
        ("row_keep_kv", C.POINTER(C.c_int32)),
    ]


class SynthParams(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("n_spans", C.c_uint32),
        ("n_points", C.c_uint32),
        ("t0", C.c_uint32),
        ("step", C.c_uint32),
        ("kind", C.c_uint32),
        ("span0", C.c_uint32),
    ]


def ptr(arr, ctype):
    """numpy array -> ctypes pointer (array must stay alive)."""
    return arr.ctypes.data_as(C.POINTER(ctype))
