"""The goldens through TEMPI with ONE HIP runtime, torch's: torch is imported
before libtempi is loaded, so its bundled libamdhip64.so (SONAME
libamdhip64.so.7) satisfies libtempi_hip.so and no second runtime is mapped
-- the configuration bench.py and smoke() run in, while the pytest process
holds two. Every golden case (MPICH 3.3.2's packed bytes,
positions and unpacked buffers, tests/golden/) is packed and unpacked from
device buffers; the strided ones must take the GPU path.
usage: torch_runtime_parity.py -> "RESULT ok <n> cases" """
import ctypes
import os
import sys

import torch  # noqa: F401  (FIRST: its runtime is the process's only one)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402
from tests import golden_data as G  # noqa: E402
from tests import typezoo  # noqa: E402

NOT_STRIDED = {"zoo_hi", "zoo_hib", "hindexed_irregular", "struct_irregular"}

mpi = tempi_amd.get_mpi()
mpi.Init()
buf = ctypes.create_string_buffer(8192)
n = mpi.L.tempi_hip_runtimes(buf, 8192)
paths = buf.value.decode().split(";")
assert n == 1 and "torch" in paths[0], f"expected torch's runtime alone, got {paths}"
assert mpi.gpu_available(), "libtempi found no GPU"
dev = torch.device("cuda", 0)
checked = 0
for c in G.cases():
    t, temps, basic = typezoo.build(mpi, c["recipe"])
    try:
        src = (torch.arange(c["buflen"], dtype=torch.int64, device=dev) & 0xFF).to(torch.uint8)
        out = torch.zeros(max(c["pack_size"], 1), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        before = mpi.counters()
        pos = mpi.Pack(src.data_ptr() + c["origin"], c["count"], t, out.data_ptr(), c["pack_size"], 0)
        after = mpi.counters()
        assert pos == c["position"], c["name"]
        G.check_packed(c, out[:pos].cpu().numpy())
        if c["size"] and c["count"] and c["name"] not in NOT_STRIDED:
            assert after["packs"] == before["packs"] + 1 and after["lib_packs"] == before["lib_packs"], c["name"]
        dst = torch.zeros(c["buflen"], dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        upos = mpi.Unpack(out.data_ptr(), c["pack_size"], 0, dst.data_ptr() + c["origin"], c["count"], t)
        assert upos == c["unpack_position"], c["name"]
        G.check_unpacked(c, dst.cpu().numpy())
        checked += 1
    finally:
        typezoo.free(mpi, t, temps, basic)
mpi.Finalize()
print(f"RESULT ok {checked} cases", flush=True)
