// tempi_amd/csrc/core/p2p_persistent.cpp -- persistent requests:
// MPI_Send_init / MPI_Ssend_init / MPI_Bsend_init / MPI_Rsend_init /
// MPI_Recv_init, started with MPI_Start / MPI_Startall.
//
// The reference interposes none of these, so a persistent request on a device
// object reaches a library that cannot read GPU memory (its own MPI_Isend is
// built on a persistent *library* send of the packed bytes,
// /root/reference/src/internal/async_operation.cpp:97-140, but the
// application's persistent calls are not seen). Here, while TEMPI is active
// beside a GPU, every persistent request is a TEMPI request that remembers its
// arguments. MPI_Start posts the matching non-blocking operation through the
// interposed entry points -- so a device object takes the strided transport
// (p2p::isend / p2p::irecv, with its send mode), a host send keeps the send
// order behind TEMPI sends, and a host receive recognises descriptors -- and
// the completion family completes that inner request and leaves the
// persistent one inactive: MPI_Wait / MPI_Test return its status and keep the
// handle; an inactive request completes at once with an empty status and is
// skipped like MPI_REQUEST_NULL by MPI_Testany / MPI_Waitany / MPI_Testsome.
#include "p2p_internal.hpp"

#include "counters.hpp"
#include "log.hpp"
#include "next_mpi.hpp"
#include "state.hpp"

namespace tempi {
namespace p2p {
namespace detail {

namespace {

void empty_status(MPI_Status *s) {
  if (s == MPI_STATUS_IGNORE) return;
  s->MPI_SOURCE = MPI_ANY_SOURCE;
  s->MPI_TAG = MPI_ANY_TAG;
  s->MPI_ERROR = MPI_SUCCESS;
  MPI_Status_set_elements(s, MPI_BYTE, 0);
  MPI_Status_set_cancelled(s, 0);
}

} // namespace

int persistent_count = 0;

struct PersistentOp : Op {
  bool send;
  void *buf;
  int count;
  MPI_Datatype dt; // held (the application may free its type after the init call)
  int peer, tag;
  MPI_Comm comm;
  SendMode mode;
  MPI_Request inner = MPI_REQUEST_NULL; // the started operation (TEMPI's or the library's)
  bool started = false;
  MPI_Status last{};

  PersistentOp(bool s, const void *b, int c, MPI_Datatype d, int p, int t, MPI_Comm cm, SendMode m)
      : send(s), buf(const_cast<void *>(b)), count(c), dt(hold_type(d)), peer(p), tag(t), comm(cm), mode(m) {
    done = true; // (finalize does not wait on a persistent request, only on what it started)
    empty_status(&last);
  }
  ~PersistentOp() override { // (release() frees a started inner request first)
    drop_type(dt);
    --persistent_count;
  }
  PersistentOp *persistent() override { return this; }
  void status(MPI_Status *s) const override {
    if (s != MPI_STATUS_IGNORE) *s = last;
  }

  int start() {
    if (started) return raise_error(comm, MPI_ERR_REQUEST); // already active
    int rc;
    if (!send)
      rc = MPI_Irecv(buf, count, dt, peer, tag, comm, &inner);
    else if (mode == SendMode::SYNC)
      rc = MPI_Issend(buf, count, dt, peer, tag, comm, &inner);
    else if (mode == SendMode::BUFFERED)
      rc = MPI_Ibsend(buf, count, dt, peer, tag, comm, &inner);
    else if (mode == SendMode::READY)
      rc = MPI_Irsend(buf, count, dt, peer, tag, comm, &inner);
    else
      rc = MPI_Isend(buf, count, dt, peer, tag, comm, &inner);
    if (rc == MPI_SUCCESS) {
      started = true;
      counters.persistent_starts++;
    }
    return rc;
  }
  // the inner request completed with status `st`: inactive again
  void finished(const MPI_Status &st, MPI_Status *out) {
    started = false;
    inner = MPI_REQUEST_NULL;
    last = st;
    if (out != MPI_STATUS_IGNORE) *out = st;
  }
};

} // namespace detail

using namespace detail;

int persistent_init(bool send, const void *buf, int count, MPI_Datatype dt, int peer, int tag, MPI_Comm comm,
                    SendMode mode, MPI_Request *req) {
  *req = add(std::unique_ptr<Op>(new PersistentOp(send, buf, count, dt, peer, tag, comm, mode)));
  ++persistent_count;
  return MPI_SUCCESS;
}

int start(MPI_Request *req) {
  Op *op = find_op(*req);
  PersistentOp *p = op ? op->persistent() : nullptr;
  if (!p) {
    LOG_ERROR("MPI_Start on a request that is not persistent");
    return MPI_ERR_REQUEST;
  }
  return p->start();
}

bool inactive(MPI_Request r) {
  Op *op = find_op(r);
  PersistentOp *p = op ? op->persistent() : nullptr;
  return p && !p->started;
}

namespace detail {

int persistent_wait(PersistentOp *p, MPI_Status *status) {
  if (!p->started) {
    empty_status(status);
    return MPI_SUCCESS;
  }
  MPI_Status st;
  empty_status(&st);
  const int rc = MPI_Wait(&p->inner, &st);
  p->finished(st, status);
  return rc;
}

int persistent_test(PersistentOp *p, int *flag, MPI_Status *status) {
  if (!p->started) {
    *flag = 1;
    empty_status(status);
    return MPI_SUCCESS;
  }
  MPI_Status st;
  empty_status(&st);
  const int rc = MPI_Test(&p->inner, flag, &st);
  // an error before the inner request completed: that request is let go
  // (it finishes in the background) and the persistent one is inactive again
  if (rc != MPI_SUCCESS && !*flag && p->inner != MPI_REQUEST_NULL) MPI_Request_free(&p->inner);
  if (*flag || rc != MPI_SUCCESS) p->finished(st, status);
  return rc;
}

bool persistent_peek(PersistentOp *p) {
  if (!p->started) return true;
  int flag = 0;
  MPI_Request_get_status(p->inner, &flag, MPI_STATUS_IGNORE);
  return flag != 0;
}

int persistent_get_status(PersistentOp *p, int *flag, MPI_Status *status) {
  if (!p->started) {
    *flag = 1;
    empty_status(status);
    return MPI_SUCCESS;
  }
  return MPI_Request_get_status(p->inner, flag, status);
}

int persistent_cancel(PersistentOp *p) { return p->started ? MPI_Cancel(&p->inner) : MPI_SUCCESS; }

void persistent_free(PersistentOp *p) {
  if (p->started && p->inner != MPI_REQUEST_NULL) MPI_Request_free(&p->inner); // finishes in the background
  p->started = false;
}

} // namespace detail
} // namespace p2p
} // namespace tempi
