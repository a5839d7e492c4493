#!/bin/bash
# Round 3's unmeasured opt-in paths, in one call: the AQL dispatch session
# (tools/gpu_aql_session.sh: probe, syncbench, its GPU test, config-1 A/B,
# persistent-request tests), the dense-window ratio A/B
# (tools/gpu_dense_ab.sh) and the halo pre-gather A/B
# (tools/gpu_pregather_ab.sh). Stops at the first failing step.
cd "$(dirname "$0")/.."
bash tools/gpu_aql_session.sh && bash tools/gpu_dense_ab.sh && bash tools/gpu_pregather_ab.sh
