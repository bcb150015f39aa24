"""ctypes binding of ``libruleset_hip.so`` (C ABI: ``include/ruleset_hip.h``).

The library is built in-tree (``csrc/Makefile`` or ``__graft_entry__.build()``)
and loaded from ``ruleset-analysis_amd/_build/libruleset_hip.so`` only.  There
is no fallback: if the library or a symbol is missing, ``load()`` raises
``NativeUnavailable`` and every product entry point fails with it.
"""

import ctypes
import os

__all__ = ['load', 'lib_path', 'NativeUnavailable', 'NativeError', 'SYMBOLS', 'Ctx', 'Transport', 'ShardBatch',
           'MergeInfo']

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, '_build')


def lib_path():
    return os.environ.get('RSA_HIP_LIB') or os.path.join(_BUILD, 'libruleset_hip.so')


class NativeUnavailable(RuntimeError):
    pass


class NativeError(RuntimeError):
    def __init__(self, code, msg):
        RuntimeError.__init__(self, 'libruleset_hip error %d: %s' % (code, msg))
        self.code = code


RSA_OK, RSA_ERR_ARG, RSA_ERR_HIP, RSA_ERR_STATE, RSA_ERR_CAPACITY = 0, -1, -2, -3, -4
RSA_OPT_AUTO_FILTER, RSA_OPT_USE_INDEX, RSA_OPT_PROFILE_SKIP, RSA_OPT_FILTER_SLICE, RSA_OPT_FILTER_STEPS = 1, 2, 3, 5, 7
RSA_OPT_FORCE_DEFER = 8
RSA_OPT_PRECHECK = 9
RSA_OPT_STATS = 10
RSA_OPT_WAVE_CAP_SCATTER = 11
RSA_OPT_GROUP_TASKS = 12
RSA_OPT_PROFILE_CLASSIFY = 13
RSA_OPT_HOT_SPLIT, RSA_OPT_HOT_MIN, RSA_OPT_PARSE_STAGED, RSA_OPT_REGION_IMPORT = 14, 15, 16, 17
RSA_OPT_COUNT_SORT, RSA_OPT_OWNER_WORLD, RSA_OPT_OWNER_RANK, RSA_OPT_MIN_REGIONS_LOG2 = 18, 19, 20, 21
RSA_OPT_REGION_RECORDS, RSA_OPT_REDUCE_BIG, RSA_OPT_FILTER_GROWTH = 22, 23, 24
RSA_OPT_COUNTER_WORDS16, RSA_OPT_CLASSIFY_PAIR = 26, 28
RSA_OPT_ROUTE_ROWS = 29

P = ctypes.c_void_p
U32 = ctypes.c_uint32
U64 = ctypes.c_uint64
I32 = ctypes.c_int
PU32 = ctypes.POINTER(ctypes.c_uint32)
PU64 = ctypes.POINTER(ctypes.c_uint64)

RSA_MERGE_GATHER, RSA_MERGE_ALWAYS_EXCHANGE = 1, 2

# rsa_transport callbacks: all_reduce_i64(self, buf, n, op, stream), all_to_allv(self, send, send_bytes, recv,
# recv_bytes, stream)
ALL_REDUCE_FN = ctypes.CFUNCTYPE(I32, P, ctypes.POINTER(ctypes.c_int64), U64, I32, P)
ALL_TO_ALLV_FN = ctypes.CFUNCTYPE(I32, P, P, PU64, P, PU64, P)


class Transport(ctypes.Structure):
    _fields_ = [('self', P), ('world', ctypes.c_int32), ('rank', ctypes.c_int32), ('host_buffers', ctypes.c_int32),
                ('all_reduce_i64', ALL_REDUCE_FN), ('all_to_allv', ALL_TO_ALLV_FN)]


class ShardBatch(ctypes.Structure):
    _fields_ = [('d_tuples', P), ('d_ts', P), ('d_order', P), ('d_gid', P), ('n', U64)]


class MergeInfo(ctypes.Structure):
    _fields_ = [('d_rows', P), ('n_rows', U64), ('owner_rows', U64), ('gather_rows', U64),
                ('route1_sent', U64), ('route1_self', U64), ('route1_recv', U64),
                ('route2_sent', U64), ('route2_self', U64), ('route2_recv', U64),
                ('allreduce_bytes', U64), ('needed', U64), ('reexports', U32), ('pass2', U32)]

# name -> (restype, argtypes); exactly the functions declared in include/ruleset_hip.h
SYMBOLS = {
    'rsa_version': (I32, []),
    'rsa_ctx_create': (I32, [I32, ctypes.POINTER(P)]),
    'rsa_ctx_destroy': (I32, [P]),
    'rsa_last_error': (ctypes.c_char_p, [P]),
    'rsa_set_stream': (I32, [P, P]),
    'rsa_set_option': (I32, [P, I32, ctypes.c_int64]),
    'rsa_load_index': (I32, [P, P, U32, P, U32]),
    'rsa_last_pass1_ms': (I32, [P, ctypes.POINTER(ctypes.c_float)]),
    'rsa_last_pass1_times': (I32, [P, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    'rsa_last_pass1_launches': (I32, [P, ctypes.POINTER(ctypes.c_uint32)]),
    'rsa_load_rules': (I32, [P, P, U32, P, U32, U32]),
    'rsa_bind_counters': (I32, [P, P, P, P, P]),
    'rsa_set_rule_count': (I32, [P, U32]),
    'rsa_reset': (I32, [P, U64, U32]),
    'rsa_classify': (I32, [P, P, P, P, U64, P]),
    'rsa_classify_only': (I32, [P, P, U64, P]),
    'rsa_aggregate_gids': (I32, [P, P, P, P, P, U64]),
    'rsa_resolve_cap': (I32, [P, PU32]),
    'rsa_recount': (I32, [P, P, P, P, P, U64]),
    'rsa_emit': (I32, [P, P, U64, PU64]),
    'rsa_table_size': (I32, [P, PU64]),
    'rsa_stats': (I32, [P, PU64, I32]),
    'rsa_export': (I32, [P, I32, P, U64, PU64]),
    'rsa_export_routed': (I32, [P, I32, U32, P, U64, P]),
    'rsa_import': (I32, [P, I32, P, U64]),
    'rsa_merge': (I32, [P, ctypes.POINTER(Transport), P, U32, I32, ctypes.POINTER(MergeInfo)]),
    'rsa_gather': (I32, [P, ctypes.POINTER(Transport), ctypes.POINTER(MergeInfo)]),
    'rsa_merge_rows': (I32, [P, I32, P, U64, PU64]),
    'rsa_rccl_unique_id': (I32, [P]),
    'rsa_rccl_comm_create': (I32, [P, ctypes.c_int32, ctypes.c_int32, P, ctypes.POINTER(P)]),
    'rsa_rccl_comm_destroy': (I32, [P]),
    'rsa_merge_rccl': (I32, [P, P, P, U32, I32, ctypes.POINTER(MergeInfo)]),
    'rsa_gather_rccl': (I32, [P, P, ctypes.POINTER(MergeInfo)]),
    'rsa_shadowed': (I32, [P, P, U32, P]),
    'rsa_shadowed_ports': (I32, [P, P, U32, P, U32, P]),
    'rsa_text_count_lines': (I32, [P, P, U64, PU64]),
    'rsa_text_line_offsets': (I32, [P, P, U64, P, U64]),
    'rsa_text_split': (I32, [P, P, U64, P, U64, PU64]),
    'rsa_parse_text': (I32, [P, P, P, U64, P, U32, P, U32, P, P, P]),
    'rsa_order_keys': (I32, [P, P, P, U64, U64, P]),
    'rsa_order_keys_grouped': (I32, [P, P, P, U64, P, U64, P]),
    'rsa_parse_reduce': (I32, [P, P, P, U64, P, U32, P, P, P]),
    'rsa_sync': (I32, [P]),
}

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise NativeUnavailable('libruleset_hip.so not built (%s); run __graft_entry__.build() or make -C '
                                'ruleset-analysis_amd/csrc' % path)
    try:
        lib = ctypes.CDLL(path)
    except OSError as exc:
        raise NativeUnavailable('cannot load %s: %s' % (path, exc))
    for name, (res, args) in SYMBOLS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            raise NativeUnavailable('%s does not export %s' % (path, name))
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class Ctx(object):
    """Owns one rsa_ctx; raises NativeError on any non-zero status."""

    def __init__(self, device=0):
        self.lib = load()
        h = P()
        rc = self.lib.rsa_ctx_create(int(device), ctypes.byref(h))
        if rc != RSA_OK:
            raise NativeError(rc, 'rsa_ctx_create(device=%d) failed' % device)
        self.h = h
        self.device = device

    def check(self, rc, what):
        if rc != RSA_OK:
            msg = self.lib.rsa_last_error(self.h)
            raise NativeError(rc, '%s: %s' % (what, msg.decode() if msg else ''))

    def call(self, name, *args):
        self.check(getattr(self.lib, name)(self.h, *args), name)

    def close(self):
        if self.h:
            self.lib.rsa_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass
