"""Helpers to launch MPI programs (MPICH's mpiexec, /opt/conda). The whole
process group is killed on timeout, so no rank outlives a hung test."""
import os
import signal
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
MPIEXEC = os.environ.get("TEMPI_MPIEXEC", "/opt/conda/bin/mpiexec")


def run(n, argv, env=None, timeout=240):
    e = dict(os.environ)
    e.update(env or {})
    e.setdefault("HYDRA_LAUNCHER", "fork")
    cmd = [MPIEXEC, "-n", str(n)] + argv
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=e, cwd=ROOT,
                         start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, _ = p.communicate()
        return -9, (out or "") + f"\n[mpi_launch] killed after {timeout} s"
    return p.returncode, out


def py(script, *args):
    return [sys.executable, "-u", os.path.join(ROOT, "tests", "mpi_progs", script)] + list(args)
