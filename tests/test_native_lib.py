"""The C-ABI library builds for gfx950, loads, and exports every entry point
declared in include/ruleset_hip.h (no compute calls: no GPU needed)."""
import ctypes
import os
import re

from conftest import ROOT
from ruleset_analysis_amd import native


def _declared():
    with open(os.path.join(ROOT, 'include', 'ruleset_hip.h')) as f:
        src = f.read()
    return sorted(set(re.findall(r'^(?:int|const char \*|void)\s*\*?\s*(rsa_\w+)\s*\(', src, re.M)))


def test_header_and_binding_agree():
    assert _declared() == sorted(native.SYMBOLS)


def test_library_exports_all_symbols():
    lib = native.load()
    for name in _declared():
        assert hasattr(lib, name), name
    assert lib.rsa_version() == 2


def test_library_is_gfx950_code_object():
    with open(native.lib_path(), 'rb') as f:
        blob = f.read()
    assert b'gfx950' in blob


def test_struct_layouts():
    from ruleset_analysis_amd.compile import RECORD_DTYPE, RULE_DTYPE, TUPLE_DTYPE
    assert (TUPLE_DTYPE.itemsize, RULE_DTYPE.itemsize, RECORD_DTYPE.itemsize) == (16, 32, 40)


def test_ctx_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        return
    lib = native.load()
    h = ctypes.c_void_p()
    assert lib.rsa_ctx_create(0, ctypes.byref(h)) != 0


def test_no_signed_mul24_shifts():
    """HIP's __umul24 returns a signed int: shifting a product >= 2^31 right
    sign-extends it (an index of a table with more than 2^15 slots or buckets
    went negative and faulted).  Only the unsigned wrapper may call it."""
    for name in ('ruleset_hip.hip', 'textparse.hip', 'textparse_line.h'):
        with open(os.path.join(ROOT, 'ruleset-analysis_amd', 'csrc', name)) as f:
            calls = [l for l in f if '__umul24(' in l and 'uint32_t umul24(' not in l and not l.lstrip().startswith('//')]
        assert calls == [], (name, calls)


def test_header_constants_equal_binding():
    """Every RSA_OPT_* / RSA_ERR_* / RSA_LINE_* / RSA_F_* / RSA_RED_* value the
    binding names equals the header's #define (the options are plain ints on
    the ctypes side)."""
    with open(os.path.join(ROOT, 'include', 'ruleset_hip.h')) as f:
        text = f.read()
    defs = {m.group(1): int(m.group(2), 0) for m in
            re.finditer(r'^#define\s+(RSA_(?:OPT|ERR|LINE|F|RED|MERGE)_[A-Z0-9_]+)\s+\(?(-?(?:0x)?[0-9A-Fa-f]+)u?\)?', text,
                        re.M)}
    bound = {k: getattr(native, k) for k in dir(native) if k in defs}
    assert len(bound) >= 20
    for k, v in bound.items():
        assert v == defs[k], k
    assert {'RSA_OPT_COUNT_SORT', 'RSA_OPT_OWNER_WORLD', 'RSA_OPT_OWNER_RANK', 'RSA_MERGE_GATHER',
            'RSA_MERGE_ALWAYS_EXCHANGE'} <= set(bound)


def test_merge_struct_layouts_equal_header(tmp_path):
    """The ctypes mirrors of rsa_transport, rsa_shard_batch and rsa_merge_info
    have the header's sizes and field offsets (gcc on the header itself)."""
    import subprocess
    structs = [('rsa_transport', native.Transport), ('rsa_shard_batch', native.ShardBatch),
               ('rsa_merge_info', native.MergeInfo)]
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "ruleset_hip.h"', 'int main(void) {']
    for cname, cls in structs:
        lines.append('printf("%%zu\\n", sizeof(%s));' % cname)
        for f, _t in cls._fields_:
            lines.append('printf("%%zu\\n", offsetof(%s, %s));' % (cname, f))
    lines.append('return 0; }')
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(lines) + '\n')
    exe = tmp_path / 'layout'
    subprocess.run(['gcc', '-I', os.path.join(ROOT, 'include'), '-o', str(exe), str(src)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = []
    for _cname, cls in structs:
        want.append(ctypes.sizeof(cls))
        want.extend(getattr(cls, f).offset for f, _t in cls._fields_)
    assert got == want
