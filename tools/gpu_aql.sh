#!/bin/bash
# HIP launch vs a hand-written AQL dispatch packet on the synchronous small
# call's critical path (tools/aqlbench.hip). gpurun_out/aql.jsonl.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 90 tools/_variants/aqlbench tools/_variants/aqlbench.hsaco 2000 > gpurun_out/aql.jsonl 2> gpurun_out/aql.err
rc=$?; cat gpurun_out/aql.err; cat gpurun_out/aql.jsonl; exit $rc
