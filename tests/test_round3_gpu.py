"""Round 3's additions on the GPU: persistent requests and the send modes on
device objects, and the transport fuzz with send modes / persistent requests
/ host receives of device sends. Every byte is checked against the oracle.
(Round 3's opt-in AQL dispatch and pre-gather were measured in round 4 --
no gain on config 1, and a slower halo -- and removed: profiles/r04/
aql_session_s2.log, pregather_ab_s2.jsonl.)"""

import pytest

from tests import mpi_launch

pytestmark = pytest.mark.gpu

METHODS = {
    "AUTO": {},
    "ONESHOT": {"TEMPI_DATATYPE_ONESHOT": "1"},
    "STAGED": {"TEMPI_DATATYPE_STAGED": "1"},
    "IPC": {"TEMPI_DATATYPE_IPC": "1"},
    "XCOPY": {"TEMPI_DATATYPE_IPC": "1", "TEMPI_IPC_COPY_MIN_BYTES": "1", "TEMPI_IPC_COPY_MIN_BLOCK": "1"},
}


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
                                        (1, 37, {"TEMPI_STREAMS": "1"})])
def test_transport_fuzz_modes(gpu, n, seed, env):
    """the transport fuzz with send modes (MPI_Issend / MPI_Ibsend), persistent
    sends and receives, and host receives of device sends mixed in; with and
    without the self channel"""
    rc, out = mpi_launch.run(n, mpi_launch.py("fuzz.py", "5", str(seed), "--modes"), env=env, timeout=200)
    assert rc == 0 and "RESULT errors=0" in out, out[-3000:]
