"""A minimal PMI-1 process manager, so that MPICH ranks can be launched by
something other than mpiexec (torch.distributed.run in bench.py).

MPICH's simple PMI client (the one its hydra launcher serves) talks a
line-oriented text protocol over a socket whose descriptor it finds in
PMI_FD; PMI_RANK / PMI_SIZE give its place. This module serves that protocol
from a thread in rank 0: init, get_maxes, get_appnum, get_my_kvsname,
get_universe_size, put / get / getbyidx on one key-value space, barrier_in /
barrier_out, finalize. "PMI_process_mapping" is pre-set to one node holding
every rank (MPICH reads it to find node-local peers for shared memory).

Usage (every rank, before MPI_Init):
    srv = pmi.Server(world) if rank == 0 else None   # rank 0 only
    port = <broadcast srv.port from rank 0>
    keep = pmi.connect(port, rank, world)            # sets PMI_FD etc.
"""
import os
import socket
import threading

KVS = "kvs_tempi_0"


class Server:
    def __init__(self, size, host="127.0.0.1"):
        self.size = size
        self.kv = {"PMI_process_mapping": f"(vector,(0,1,{size}))"}
        self.lock = threading.Lock()
        self.barrier = []
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, 0))
        self.sock.listen(size)
        self.port = self.sock.getsockname()[1]
        self.done = 0
        threading.Thread(target=self._accept, daemon=True).start()

    def _accept(self):
        for _ in range(self.size):
            c, _ = self.sock.accept()
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    def _serve(self, c):
        buf = b""
        while True:
            try:
                data = c.recv(65536)
            except OSError:
                return
            if not data:
                return
            buf += data
            while b"\n" in buf:
                line, buf = buf.split(b"\n", 1)
                if not self._handle(c, line.decode()):
                    c.close()
                    return

    def _handle(self, c, line):
        f = {}
        for tok in line.strip().split(" "):
            if "=" in tok:
                k, v = tok.split("=", 1)
                f[k] = v
        cmd = f.get("cmd", "")
        send = lambda s: c.sendall((s + "\n").encode())
        if cmd == "init":
            send("cmd=response_to_init pmi_version=1 pmi_subversion=1 rc=0")
        elif cmd == "get_maxes":
            send("cmd=maxes kvsname_max=256 keylen_max=256 vallen_max=4096 rc=0")
        elif cmd == "get_appnum":
            send("cmd=appnum appnum=0 rc=0")
        elif cmd == "get_my_kvsname":
            send(f"cmd=my_kvsname kvsname={KVS} rc=0")
        elif cmd == "get_universe_size":
            send(f"cmd=universe_size size={self.size} rc=0")
        elif cmd == "put":
            with self.lock:
                self.kv[f.get("key", "")] = f.get("value", "")
            send("cmd=put_result rc=0")
        elif cmd == "get":
            with self.lock:
                v = self.kv.get(f.get("key", ""))
            send(f"cmd=get_result rc=0 value={v}" if v is not None else "cmd=get_result rc=-1 msg=key_not_found")
        elif cmd == "getbyidx":
            send("cmd=getbyidx_results rc=-2 reason=no_more_keyvals")
        elif cmd == "barrier_in":
            with self.lock:
                self.barrier.append(c)
                if len(self.barrier) == self.size:
                    waiting, self.barrier = self.barrier, []
                    for w in waiting:
                        w.sendall(b"cmd=barrier_out rc=0\n")
        elif cmd == "finalize":
            send("cmd=finalize_ack rc=0")
            return False
        elif cmd == "abort":
            os._exit(int(f.get("exitcode", "1")))
        else:
            send(f"cmd={cmd}_result rc=-1 msg=unsupported")
        return True


def connect(port, rank, size, host="127.0.0.1"):
    """Connect this process to the server and point MPICH at the socket.
    Returns the socket, which must stay open until MPI_Finalize."""
    s = socket.create_connection((host, port))
    os.set_inheritable(s.fileno(), True)
    os.environ["PMI_FD"] = str(s.fileno())
    os.environ["PMI_RANK"] = str(rank)
    os.environ["PMI_SIZE"] = str(size)
    for k in ("PMI_PORT", "PMI_ID"):
        os.environ.pop(k, None)
    return s


def wire_torch_ranks(rank, size, dist):
    """Under torch.distributed (initialised): rank 0 serves, everyone
    connects. Returns (server_or_None, socket)."""
    srv = Server(size) if rank == 0 else None
    box = [srv.port if srv else 0]
    dist.broadcast_object_list(box, src=0)
    return srv, connect(box[0], rank, size)
