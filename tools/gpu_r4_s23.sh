#!/bin/bash
# Grid-size cap A/B (grid-stride beyond TEMPI_MAX_BLOCKS workgroups): cur (no
# cap in practice) vs 2048 / 8192 / 32768, tools/build_ab.sh builds, kernel
# times by tools/kab.sh on the headline shape and wide / narrow / 3-D ones.
cd "$(dirname "$0")/.."
bash tools/kab.sh gridcap_ab.jsonl 3 20 512:2097152:1024 4096:262144:8192 64:16777216:128 8:134217728:16 \
  24:512:2386944:512:4608 || exit 3
python3 tools/kab_summary.py gpurun_out/gridcap_ab.jsonl 2>&1 | tail -40
