"""Round 3's additions on the GPU, kept in a file of their own that runs
after the established suite: persistent requests and the send modes on
device objects, the transport fuzz with send modes / persistent requests /
host receives of device sends, the opt-in pre-gather (TEMPI_PREGATHER_BYTES)
under the fuzz and the full-size halo check, and the opt-in AQL dispatch
path (TEMPI_AQL, skipped unless TEMPI_TEST_AQL=1). Every byte is checked
against the oracle."""
import json
import os

import pytest

from tests import mpi_launch

pytestmark = pytest.mark.gpu

LIB = os.path.join(mpi_launch.ROOT, "tempi_amd", "lib")
METHODS = {
    "AUTO": {},
    "ONESHOT": {"TEMPI_DATATYPE_ONESHOT": "1"},
    "STAGED": {"TEMPI_DATATYPE_STAGED": "1"},
    "IPC": {"TEMPI_DATATYPE_IPC": "1"},
    "XCOPY": {"TEMPI_DATATYPE_IPC": "1", "TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_IPC_COPY_MIN_BLOCK": "1"},
}


def _json_line(out):
    for line in out.splitlines():
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError(out[-3000:])


@pytest.mark.parametrize("n,method", [(1, "AUTO"), (2, "AUTO"), (2, "ONESHOT"), (2, "IPC"), (2, "STAGED"),
                                      (2, "XCOPY")])
def test_persistent_and_send_modes_device(gpu, n, method):
    """device objects through persistent requests (every init call, MPI_Start /
    MPI_Startall, inactive requests in the completion family, cancel, a
    persistent host receive of a device send) and MPI_Ssend / Bsend / Rsend /
    Issend / Ibsend / Irsend; one rank sends to itself"""
    rc, out = mpi_launch.run(n, mpi_launch.py("persistent.py", "--device"), env=METHODS[method], timeout=240)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


@pytest.mark.parametrize("n,seed,env", [(1, 41, {}), (2, 43, {}), (3, 47, {}), (2, 53, {"TEMPI_NO_SELF_CHANNEL": "1"}),
                                        (2, 31, {"TEMPI_PREGATHER_BYTES": "1000000000", "TEMPI_PREGATHER_MAX_BLOCK":
                                                 "1000000", "TEMPI_PREGATHER_FLUSH": "1"}),
                                        (1, 37, {"TEMPI_PREGATHER_BYTES": "100000", "TEMPI_PREGATHER_MAX_BLOCK": "64"})])
def test_transport_fuzz_modes(gpu, n, seed, env):
    """the transport fuzz with send modes (MPI_Issend / MPI_Ibsend), persistent
    sends and receives, and host receives of device sends mixed in; with and
    without the self channel and the pre-gather"""
    rc, out = mpi_launch.run(n, mpi_launch.py("fuzz.py", "5", str(seed), "--modes"), env=env, timeout=200)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]


def test_halo_exchange_512_pregather(gpu):
    """config 4 at full size, one rank, with the pre-gather on: every cell of
    every quantity checked"""
    rc, out = mpi_launch.run(1, [os.path.join(LIB, "halo_exchange"), "2", "512", "--check"],
                             env={"TEMPI_PREGATHER_BYTES": "134217728"}, timeout=240)
    r = _json_line(out)
    assert rc == 0 and r["checked"] and r["errors"] == 0, out[-3000:]


@pytest.mark.skipif(os.environ.get("TEMPI_TEST_AQL") != "1",
                    reason="TEMPI_AQL is opt-in and not yet run on this pool's GPUs (DESIGN §6): "
                           "set TEMPI_TEST_AQL=1 (tools/gpu_aql_session.sh does)")
def test_synchronous_calls_through_aql_packets(gpu):
    """TEMPI_AQL=1: synchronous MPI_Pack / MPI_Unpack launched by TEMPI's own
    AQL dispatch packets (hip/aql.hpp), every result visible device-wide right
    after the call, and the packets really used (dispatch count: 5 of the 6
    shapes fold their ticket, 2 x 40 calls each; a kernel whose code object
    HIP has not loaded yet launches through HIP once)"""
    rc, out = mpi_launch.run(1, mpi_launch.py("aql_sync.py"), env={"TEMPI_AQL": "1"}, timeout=200)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]
    n = int(out.split("aql_dispatches=")[1].split()[0])
    assert 5 * 80 - 10 <= n <= 5 * 80, out[-3000:]
