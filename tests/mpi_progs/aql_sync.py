"""Run under mpiexec -n 1 with TEMPI_AQL=1: synchronous MPI_Pack / MPI_Unpack
between device buffers dispatched by TEMPI's own AQL packets (hip/aql.hpp)
instead of hipLaunchKernelGGL. After each call a kernel on torch's stream
compares the result (the bytes must already be visible device-wide), 40
rounds per shape with fresh contents, over shapes that take each kernel
family (16-byte words, interleaved 24-byte rows, the dense-window gather,
4-byte words, one workgroup, and a grid too large to fold, which launches
through HIP behind the queue's ticket). Prints the AQL dispatch count."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402
import torch  # noqa: E402

torch.cuda.set_device(0)
gpu = torch.device("cuda", 0)
mpi = tempi_amd.get_mpi()
mpi.Init()
errors = 0
c0 = mpi.counters()
for rows, block, stride in [(1024, 512, 1024), (4096, 24, 4608), (20000, 3, 7), (100, 500, 1000), (2, 512, 1024),
                            (16384, 512, 1024)]:
    t = mpi.Type_commit(mpi.Type_vector(rows, block, stride, mpi.BYTE))
    ext = (rows - 1) * stride + block
    src = torch.empty(ext, dtype=torch.uint8, device=gpu)
    packed = torch.empty(rows * block, dtype=torch.uint8, device=gpu)
    back = torch.zeros(ext, dtype=torch.uint8, device=gpu)
    g = torch.Generator(device=gpu).manual_seed(rows)
    idx = (torch.arange(rows, device=gpu).unsqueeze(1) * stride + torch.arange(block, device=gpu)).reshape(-1)
    for r in range(40):
        src.random_(0, 256, generator=g)
        exp = src[idx]
        torch.cuda.synchronize()
        mpi.Pack(src.data_ptr(), 1, t, packed.data_ptr(), packed.numel(), 0)
        if not torch.equal(packed, exp):
            errors += 1
            print(f"vector({rows},{block},{stride}) round {r}: packed bytes not visible", flush=True)
        back.fill_(r & 0xFF)
        torch.cuda.synchronize()
        mpi.Unpack(packed.data_ptr(), packed.numel(), 0, back.data_ptr(), 1, t)
        if not torch.equal(back[idx], exp):
            errors += 1
            print(f"vector({rows},{block},{stride}) round {r}: unpacked bytes not visible", flush=True)
    mpi.Type_free(t)
c1 = mpi.counters()
aql = c1["aql_dispatches"] - c0["aql_dispatches"]
mpi.Finalize()
print(f"RESULT errors={errors} aql_dispatches={aql}", flush=True)
sys.exit(1 if errors else 0)
