/*
 * include/tempi_mpi.h -- THE DROP-IN BOUNDARY: the MPI C entry points that
 * libtempi.so exports. An unmodified application links `-ltempi` before its
 * MPI library (or LD_PRELOADs libtempi.so); each call below is handled by
 * TEMPI when its buffers are GPU-accessible and its datatype canonicalises to
 * a strided block, and is otherwise forwarded to the next definition in the
 * link order, found with dlsym(RTLD_NEXT).
 *
 * The prototypes are the standard MPI-3 ones from <mpi.h>; the list is the
 * reference's exported set (/root/reference/include/symbols.hpp:10-174,
 * `grep 'extern "C"' /root/reference/src`) restricted to the data path, plus
 * MPI_Init_thread / MPI_Waitall / MPI_Test, which the reference does not
 * interpose but which must see TEMPI-owned requests.
 *
 *   symbol           replaces the reference's        TEMPI behaviour
 *   MPI_Init         src/init.cpp:22-65              resolve next MPI, env, GPU
 *   MPI_Init_thread  (not interposed: F8)            as MPI_Init; MULTIPLE under a lock, else <= SERIALIZED
 *   MPI_Query_thread (not interposed)                the same capped level
 *   MPI_Finalize     src/finalize.cpp:20-45          drain requests, free pools
 *   MPI_Type_commit  src/type_commit.cpp:16-114      canonicalise + cache
 *   MPI_Type_free    src/type_free.cpp:14-27         drop cache entry first
 *   MPI_Pack         src/pack.cpp:28-68              GPU gather kernel
 *   MPI_Unpack       src/unpack.cpp:20-59            GPU scatter kernel
 *   MPI_Send         src/send.cpp:12-17              pack + library send
 *   MPI_Recv         src/recv.cpp:19-44              library recv + unpack
 *   MPI_Isend        src/isend.cpp:11-16             async pack -> send
 *   MPI_Irecv        src/irecv.cpp:11-16             recv -> async unpack
 *   MPI_Wait         src/wait.cpp:11-16              progress TEMPI requests
 *   MPI_Waitall      (not interposed: F8)            progress TEMPI requests
 *   MPI_Test         (not interposed: F8)            progress TEMPI requests
 *   MPI_Testall / _Testany / _Waitany / _Testsome / _Waitsome / MPI_Request_free
 *   / MPI_Request_get_status / MPI_Cancel
 *                    (not interposed: F8)            understand TEMPI requests
 *   MPI_Sendrecv     (not interposed)                Irecv + Isend through TEMPI
 *                                                    when either side is a device object
 *   MPI_Probe / MPI_Iprobe / MPI_Mprobe / MPI_Improbe / MPI_Mrecv / MPI_Imrecv
 *                    (not interposed: the reference's senders always send
 *                    the packed bytes, sender.cpp:109,161)
 *                                                    a co-located device send that
 *                                                    travels as a descriptor is probed
 *                                                    with its payload size and received
 *                                                    as its payload, into host or device
 *                                                    memory
 *   MPI_Ssend / MPI_Bsend / MPI_Rsend / MPI_Issend / MPI_Ibsend / MPI_Irsend
 *                    (not interposed)                device objects take the TEMPI
 *                                                    transport, handing the library
 *                                                    their message with the same send
 *                                                    mode; host buffers: the library's
 *                                                    call, in send order
 *   MPI_Send_init / MPI_Ssend_init / MPI_Bsend_init / MPI_Rsend_init /
 *   MPI_Recv_init / MPI_Start / MPI_Startall
 *                    (not interposed)                with TEMPI active beside a GPU,
 *                                                    TEMPI persistent requests: each
 *                                                    start posts the interposed
 *                                                    non-blocking call; the request
 *                                                    stays, inactive, after its
 *                                                    wait / test
 *   MPI_Sendrecv_replace
 *                    (not interposed)                through MPI_Sendrecv when the
 *                                                    receive is TEMPI's; otherwise
 *                                                    forwarded (the self channel
 *                                                    spills first: matching order)
 *   MPI_Buffer_detach
 *                    (not interposed)                first waits until every buffered-
 *                                                    mode send of a device object has
 *                                                    been handed to the library (it
 *                                                    goes only after its gather)
 *   MPI_Barrier      (not interposed)                keeps TEMPI operations moving
 *                                                    while it waits (a peer may need
 *                                                    this rank's progress)
 *   MPI_Alltoallv    src/alltoallv.cpp:14-68         device-buffer alltoallv
 *   MPI_Neighbor_alltoallw  src/neighbor_alltoallw.cpp:11-18 (-> internal/
 *                    neighbor_alltoallw.cpp:19-77)   per-edge Isend/Irecv when
 *                                                    any block is on the GPU
 *   MPI_Neighbor_alltoallv  src/neighbor_alltoallv.cpp:12-24 (passthrough
 *                    there)                          same route as alltoallw
 *   MPI_Dist_graph_create_adjacent  src/dist_graph_create_adjacent.cpp:55-470
 *                    rank placement with reorder = 1 and TEMPI_PLACEMENT_
 *                    {KAHIP,METIS,RANDOM} when the communicator spans several
 *                    nodes (TEMPI's own partitioner for KAHIP/METIS); the new
 *                    communicator is built in application rank order
 *   MPI_Dist_graph_neighbors        src/dist_graph_neighbors.cpp:13-49
 *   MPI_Comm_rank    src/comm_rank.cpp:13-27         these two forward
 *                    unchanged: the placed communicator's library ranks are
 *                    the application's, so there is nothing to translate
 *   MPI_Comm_free    src/comm_free.cpp:13-19         drop per-handle caches
 *
 * Error behaviour: return codes of the library pass through unchanged. Where
 * TEMPI itself detects an error (a pack that does not fit in outsize, a
 * message larger than the receive that TEMPI carried) it raises
 * MPI_ERR_TRUNCATE on the communicator's error handler and returns it, with
 * the status's MPI_ERROR set (the reference silently overruns). GPU runtime failures abort with a
 * message, as the reference does (/root/reference/include/cuda_runtime.hpp:13-20).
 */
#ifndef TEMPI_MPI_H
#define TEMPI_MPI_H

#include <mpi.h>

#ifdef __cplusplus
extern "C" {
#endif

int MPI_Init(int *argc, char ***argv);
int MPI_Init_thread(int *argc, char ***argv, int required, int *provided);
int MPI_Query_thread(int *provided);
int MPI_Finalize(void);
int MPI_Type_commit(MPI_Datatype *datatype);
int MPI_Type_free(MPI_Datatype *datatype);
int MPI_Pack(const void *inbuf, int incount, MPI_Datatype datatype, void *outbuf, int outsize,
             int *position, MPI_Comm comm);
int MPI_Unpack(const void *inbuf, int insize, int *position, void *outbuf, int outcount,
               MPI_Datatype datatype, MPI_Comm comm);
int MPI_Send(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Recv(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
             MPI_Status *status);
int MPI_Isend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
              MPI_Request *request);
int MPI_Irecv(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
              MPI_Request *request);
int MPI_Wait(MPI_Request *request, MPI_Status *status);
int MPI_Waitall(int count, MPI_Request array_of_requests[], MPI_Status array_of_statuses[]);
int MPI_Test(MPI_Request *request, int *flag, MPI_Status *status);
int MPI_Testall(int count, MPI_Request array_of_requests[], int *flag, MPI_Status array_of_statuses[]);
int MPI_Testany(int count, MPI_Request array_of_requests[], int *index, int *flag, MPI_Status *status);
int MPI_Waitany(int count, MPI_Request array_of_requests[], int *index, MPI_Status *status);
int MPI_Testsome(int incount, MPI_Request array_of_requests[], int *outcount, int array_of_indices[],
                 MPI_Status array_of_statuses[]);
int MPI_Waitsome(int incount, MPI_Request array_of_requests[], int *outcount, int array_of_indices[],
                 MPI_Status array_of_statuses[]);
int MPI_Request_free(MPI_Request *request);
int MPI_Request_get_status(MPI_Request request, int *flag, MPI_Status *status);
int MPI_Cancel(MPI_Request *request);
int MPI_Sendrecv(const void *sendbuf, int sendcount, MPI_Datatype sendtype, int dest, int sendtag, void *recvbuf,
                 int recvcount, MPI_Datatype recvtype, int source, int recvtag, MPI_Comm comm, MPI_Status *status);
int MPI_Probe(int source, int tag, MPI_Comm comm, MPI_Status *status);
int MPI_Iprobe(int source, int tag, MPI_Comm comm, int *flag, MPI_Status *status);
int MPI_Mprobe(int source, int tag, MPI_Comm comm, MPI_Message *message, MPI_Status *status);
int MPI_Improbe(int source, int tag, MPI_Comm comm, int *flag, MPI_Message *message, MPI_Status *status);
int MPI_Mrecv(void *buf, int count, MPI_Datatype datatype, MPI_Message *message, MPI_Status *status);
int MPI_Imrecv(void *buf, int count, MPI_Datatype datatype, MPI_Message *message, MPI_Request *request);
int MPI_Ssend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Bsend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Rsend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm);
int MPI_Issend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
               MPI_Request *request);
int MPI_Ibsend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
               MPI_Request *request);
int MPI_Irsend(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
               MPI_Request *request);
int MPI_Send_init(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                  MPI_Request *request);
int MPI_Ssend_init(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                   MPI_Request *request);
int MPI_Bsend_init(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                   MPI_Request *request);
int MPI_Rsend_init(const void *buf, int count, MPI_Datatype datatype, int dest, int tag, MPI_Comm comm,
                   MPI_Request *request);
int MPI_Recv_init(void *buf, int count, MPI_Datatype datatype, int source, int tag, MPI_Comm comm,
                  MPI_Request *request);
int MPI_Start(MPI_Request *request);
int MPI_Startall(int count, MPI_Request array_of_requests[]);
int MPI_Sendrecv_replace(void *buf, int count, MPI_Datatype datatype, int dest, int sendtag, int source,
                         int recvtag, MPI_Comm comm, MPI_Status *status);
int MPI_Buffer_detach(void *buffer_addr, int *size);
int MPI_Barrier(MPI_Comm comm);
int MPI_Alltoallv(const void *sendbuf, const int sendcounts[], const int sdispls[],
                  MPI_Datatype sendtype, void *recvbuf, const int recvcounts[], const int rdispls[],
                  MPI_Datatype recvtype, MPI_Comm comm);
int MPI_Neighbor_alltoallw(const void *sendbuf, const int sendcounts[], const MPI_Aint sdispls[],
                           const MPI_Datatype sendtypes[], void *recvbuf, const int recvcounts[],
                           const MPI_Aint rdispls[], const MPI_Datatype recvtypes[], MPI_Comm comm);
int MPI_Neighbor_alltoallv(const void *sendbuf, const int sendcounts[], const int sdispls[],
                           MPI_Datatype sendtype, void *recvbuf, const int recvcounts[],
                           const int rdispls[], MPI_Datatype recvtype, MPI_Comm comm);
int MPI_Dist_graph_create_adjacent(MPI_Comm comm_old, int indegree, const int sources[],
                                   const int sourceweights[], int outdegree,
                                   const int destinations[], const int destweights[],
                                   MPI_Info info, int reorder, MPI_Comm *comm_dist_graph);
int MPI_Dist_graph_neighbors(MPI_Comm comm, int maxindegree, int sources[], int sourceweights[],
                             int maxoutdegree, int destinations[], int destweights[]);
int MPI_Comm_rank(MPI_Comm comm, int *rank);
int MPI_Comm_free(MPI_Comm *comm);

#ifdef __cplusplus
}
#endif
#endif
