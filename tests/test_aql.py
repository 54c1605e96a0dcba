"""Dispatch queues (crane_queue_*, crane_dyn_step_keys_queue; csrc/aql.cpp).

CPU: the library exports the queue entry points, and every kernel in the library's code objects
takes its code-object-v5 implicit arguments where aql_launch writes them (the 8-byte aligned end
of the explicit arguments + the fixed offsets below) and no implicit argument aql_launch leaves
zero that the kernel would need.  GPU (test_aql_gpu.py): steps on a queue equal steps on a stream
and the oracle.
"""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "crane-scheduler_amd", "lib", "libcrane_dyn.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# aql_launch's implicit-argument image, relative to the aligned end of the explicit arguments
WRITTEN = {"hidden_block_count_x": 0, "hidden_block_count_y": 4, "hidden_block_count_z": 8,
           "hidden_group_size_x": 12, "hidden_group_size_y": 14, "hidden_group_size_z": 16,
           "hidden_remainder_x": 18, "hidden_remainder_y": 20, "hidden_remainder_z": 22,
           "hidden_global_offset_x": 40, "hidden_global_offset_y": 48, "hidden_global_offset_z": 56,
           "hidden_grid_dims": 64, "hidden_dynamic_lds_size": 120}


def _code_objects(tmp_path):
    """The gfx950 code objects of every offload bundle in the library's .hip_fatbin."""
    fat = tmp_path / "lib.fatbin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB, str(tmp_path / "copy.so")],
                   check=True, capture_output=True)
    data = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for i, s in enumerate(starts):
        e = starts[i + 1] if i + 1 < len(starts) else len(data)
        b = tmp_path / f"b{i}.bundle"
        b.write_bytes(data[s:e])
        co = tmp_path / f"b{i}.co"
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and co.exists() and co.stat().st_size > 0:
            out.append(co)
    return out


def _kernels(co):
    """[(symbol, [(offset, size, value_kind), ...], kernarg_segment_size)] from the code object's notes."""
    text = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                          text=True).stdout
    ks = []
    args, cur = [], {}
    for line in text.splitlines():
        t = line.strip()
        m = re.match(r"-?\s*\.(offset|size|value_kind|kernarg_segment_size|symbol):\s*(\S+)", t)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k in ("offset", "size", "value_kind"):
            if t.startswith("-") and cur:
                args.append(cur)
                cur = {}
            cur[k] = v
        elif k == "kernarg_segment_size":
            if cur:
                args.append(cur)
                cur = {}
            ks.append([None, [(int(a["offset"]), int(a["size"]), a["value_kind"]) for a in args], int(v)])
            args = []
        elif k == "symbol" and ks and ks[-1][0] is None:
            ks[-1][0] = v
    return ks


needs_tools = pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(f"{LLVM}/clang-offload-bundler")
                                      and shutil.which("true")), reason="library or ROCm LLVM tools missing")


@needs_tools
def test_implicit_arguments_where_aql_writes_them(tmp_path):
    cos = _code_objects(tmp_path)
    assert cos, "no gfx950 code object in the library"
    seen = 0
    for co in cos:
        for sym, args, seg in _kernels(co):
            if not sym or not sym.startswith("_ZN5crane"):
                continue
            seen += 1
            explicit = [a for a in args if not a[2].startswith("hidden_")]
            hidden = [a for a in args if a[2].startswith("hidden_")]
            end = max((o + s for o, s, _ in explicit), default=0)
            base = (end + 7) & ~7
            for o, s, kind in hidden:
                assert kind in WRITTEN, f"{sym}: implicit argument {kind} is not written by aql_launch"
                assert o == base + WRITTEN[kind], f"{sym}: {kind} at {o}, aql_launch writes {base + WRITTEN[kind]}"
            assert seg <= 4096, f"{sym}: kernarg segment {seg} B > the queue's 4 KiB slot"
    assert seen >= 20, f"only {seen} library kernels found in the code objects"


def test_queue_symbols_exported():
    lib = ctypes.CDLL(LIB)
    for name in ("crane_queue_create", "crane_queue_wait", "crane_queue_last_error", "crane_queue_destroy",
                 "crane_dyn_step_keys_queue"):
        assert hasattr(lib, name), name
