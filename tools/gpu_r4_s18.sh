#!/bin/bash
# A/B of a batch-launch change (cur) against the commit before ($1; round 4
# used it for one-item batches through the single-object kernel, s18, and for
# the 8-slot argument block of small batches, s24): tools/smallbatch at the C ABI, config 3's
# small strided ping-pong (pingpong_nd, 1 KiB, 8-byte rows at stride 512) and
# the reference's bench_mpi_isend pattern (1 B, 64 KiB; 1 and 10 tags), 2
# ranks on the one GPU, content-checked, three rounds with the order rotated.
# Builds: tools/build_ab.sh $1, copied to tools/_variants/ld_<v>/libtempi_hip.so.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
P=$1
O=gpurun_out; mkdir -p $O; : > $O/single_item_ab.jsonl
one() { # variant round
  local L=$PWD/tools/_variants/ld_$1
  LD_LIBRARY_PATH=$L timeout -k 10 60 tools/_variants/smallbatch 1000 | sed "s/^{/{\"variant\": \"$1\", \"round\": $2, /" >> $O/single_item_ab.jsonl || exit 3
  LD_LIBRARY_PATH=$L timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 300 1024 8 512 --check 2>/dev/null \
    | grep '^{' | sed "s/^{/{\"variant\": \"$1\", \"round\": $2, \"bench\": \"pingpong_nd\", /" >> $O/single_item_ab.jsonl || exit 4
  LD_LIBRARY_PATH=$L timeout -k 10 120 /opt/conda/bin/mpiexec -n 8 tempi_amd/lib/alltoallv_sparse 20 --scale 1000 --density 0.5 --check 2>/dev/null \
    | grep '^{' | sed "s/^{/{\"variant\": \"$1\", \"round\": $2, \"bench\": \"alltoallv\", /" >> $O/single_item_ab.jsonl || exit 6
  for t in 1 10; do
    LD_LIBRARY_PATH=$L timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/mpi_isend 200 1 65536 --tags $t --check 2>/dev/null \
      | grep '^{' | sed "s/^{/{\"variant\": \"$1\", \"round\": $2, \"bench\": \"mpi_isend\", /" >> $O/single_item_ab.jsonl || exit 5
  done
}
r=0
for order in "cur $P" "$P cur" "cur $P"; do
  r=$((r + 1))
  for v in $order; do one $v $r; done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/single_item_ab.jsonl"):
    x = json.loads(l)
    if x.get("bench") == "smallbatch":
        k = (x["dir"], x["packed"], x["shape"]); v = x["call_us"]
    elif x.get("bench") == "alltoallv":
        k = ("alltoallv8", x.get("scale"), x.get("errors")); v = x["min_us"]
    elif x.get("bench") == "pingpong_nd":
        k = ("pingpong_nd", x.get("total"), x.get("errors")); v = x["oneway_us"]
    else:
        k = ("mpi_isend", x["bytes"], x["tags"], x["errors"]); v = x["roundtrip_us"]
    d[(k, x["variant"])].append(v)
for (k, var), v in sorted(d.items(), key=lambda t: (str(t[0][0]), t[0][1])):
    print(k, var, [round(a, 2) for a in v])
PY
