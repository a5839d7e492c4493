set -o pipefail
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O
FOCUS="torch_runtime_only or probe_holds" bash tools/gpu_session.sh focus || exit 1
: > $O/soak_r6.txt
for m in "" "TEMPI_DATATYPE_ONESHOT=1" "TEMPI_DATATYPE_DEVICE=1"; do
  for n in 1 2 4; do
    env $m timeout -k 10 300 /opt/conda/bin/mpiexec -n $n python -u tests/mpi_progs/threads.py MULTIPLE MULTIPLE 6 300 --device --concurrent > $O/soak.log 2>&1
    rc=$?; echo "threads n=$n env=${m:-AUTO} rc=$rc $(grep -o 'RESULT errors=[0-9]*' $O/soak.log | sort | uniq -c | tr '\n' ' ')" | tee -a $O/soak_r6.txt
    [ $rc -eq 0 ] || exit 1
  done
done
timeout -k 10 300 /opt/conda/bin/mpiexec -n 2 python -u tests/mpi_progs/probe_threads.py 1000 > $O/soak.log 2>&1
rc=$?; echo "probe_threads n=2 rounds=1000 rc=$rc $(grep -o 'RESULT errors=[0-9]*' $O/soak.log | sort | uniq -c | tr '\n' ' ')" | tee -a $O/soak_r6.txt
[ $rc -eq 0 ] || exit 1
bash tools/transport_fuzz_wide.sh 5 10 | tail -3
