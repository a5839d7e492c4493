"""The AQL dispatch path (tempi_amd/csrc/hip/aql.hip, TEMPI_AQL=1) writes a
kernel's arguments itself: the explicit ones as the host lays out (A a,
Sig sg), then code object v5's implicit block, of which it fills the block
counts, group sizes and grid dims. Checked here without a GPU, against the
metadata of the code object actually built into libtempi_hip.so (extracted
with the ROCm LLVM tools): for every kernel the path may dispatch, the two
explicit arguments sit where the host puts them, the implicit block starts
8-byte aligned right behind them, its fields sit at the offsets aql.hip
writes, nothing else implicit is asked for, and the argument segment is
exactly explicit + 256 bytes (aql.hip refuses any other size)."""
import ctypes
import os
import re
import shutil
import subprocess

import pytest

import tempi_amd

LLVM = "/opt/rocm/lib/llvm/bin"
# what aql.hip fills (relative to the implicit block), and what it may leave 0
FILLED = {"hidden_block_count_x": 0, "hidden_group_size_x": 12, "hidden_grid_dims": 64}
ZERO_OK = {"hidden_block_count_y", "hidden_block_count_z", "hidden_group_size_y", "hidden_group_size_z",
           "hidden_remainder_x", "hidden_remainder_y", "hidden_remainder_z", "hidden_global_offset_x",
           "hidden_global_offset_y", "hidden_global_offset_z"}
# (aql.hip also writes 1 into the y / z counts and sizes: checked at their offsets)
ONES = {"hidden_block_count_y": 4, "hidden_block_count_z": 8, "hidden_group_size_y": 14,
        "hidden_group_size_z": 16}
KERNEL = re.compile(r"_ZN12_GLOBAL__N_1\d+(pack_kernel|unpack_kernel|pack_il_kernel|unpack_il_kernel|"
                    r"pack_dense_kernel)I(?:Li(\d+)E)?Li(\d+)EE")


def _tools():
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler",
                                                               "llvm-readelf"))


def _kernels(tmp_path):
    fat, co = tmp_path / "fat.bin", tmp_path / "dev.co"
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", tempi_amd.LIBTEMPI_HIP,
                    str(tmp_path / "stripped.so")], check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                   check=True, capture_output=True)
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", str(co)], check=True,
                           capture_output=True, text=True).stdout
    kernels, cur, arg, in_args = [], None, None, False
    for line in notes.splitlines():
        if line.startswith("  - .agpr_count:"):
            cur = {"args": []}
            kernels.append(cur)
            in_args = False
            continue
        if cur is None:
            continue
        if line.startswith("    .args:"):
            in_args = True
            continue
        if in_args and line.startswith("      - ."):
            arg = {}
            cur["args"].append(arg)
            line = "        " + line[8:]
        if in_args and line.startswith("        ."):
            k, _, v = line.strip().partition(":")
            arg[k[1:]] = v.strip()
            continue
        if line.startswith("    .") and not line.startswith("      "):
            in_args = False
            k, _, v = line.strip().partition(":")
            cur[k[1:]] = v.strip()
    return kernels


@pytest.mark.skipif(not _tools(), reason="ROCm LLVM tools not found")
def test_aql_kernarg_layout_matches_code_object(tmp_path):
    H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
    H.tempi_hip_aql_arg_bytes.restype = ctypes.c_int64
    seen = 0
    for k in _kernels(tmp_path):
        m = KERNEL.match(k.get("name", ""))
        if not m:
            continue
        seen += 1
        nd = int(m.group(3))
        name = k["name"]
        args = k["args"]
        explicit = [a for a in args if a["value_kind"] == "by_value"]
        assert len(explicit) == 2 and int(explicit[0]["offset"]) == 0, name
        end = int(explicit[1]["offset"]) + int(explicit[1]["size"])
        assert int(explicit[1]["size"]) == 56, name  # tempi_ticket::Sig
        assert end == H.tempi_hip_aql_arg_bytes(nd), (name, end, H.tempi_hip_aql_arg_bytes(nd))
        base = (end + 7) & ~7
        hidden = {a["value_kind"]: int(a["offset"]) - base for a in args if a["value_kind"].startswith("hidden_")}
        for kind, at in FILLED.items():
            assert hidden.get(kind) == at, (name, kind, hidden.get(kind))
        for kind, at in ONES.items():
            if kind in hidden:
                assert hidden[kind] == at, (name, kind)
        assert set(hidden) <= set(FILLED) | ZERO_OK, (name, set(hidden) - set(FILLED) - ZERO_OK)
        assert int(k["kernarg_segment_size"]) == base + 256, (name, k["kernarg_segment_size"], base)
        assert int(k["kernarg_segment_size"]) <= 1024, name  # aql.hip's kernarg slot
    assert seen >= 40, seen  # every (word width, rank) instance of the single-object kernels
