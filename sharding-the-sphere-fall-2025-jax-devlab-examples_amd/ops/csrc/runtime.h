// Native step runtime (C ABI): an op list for one integrator period, executed
// eagerly or captured once into a hipGraph and replayed.  Owns the RCCL
// communicator used for halo P2P and a high-priority comm stream.
#pragma once
#include "stsp_kernels.h"

extern "C" {

enum StspOpType { STSP_OP_STAGE = 1, STSP_OP_PACK = 2, STSP_OP_COMM_START = 3, STSP_OP_COMM_WAIT = 4,
                  STSP_OP_FUSED = 5, STSP_OP_IPC_SEND = 6, STSP_OP_IPC_WAIT = 7,
                  STSP_OP_MARCH3 = 8 };

#define STSP_MAX_PEERS 32

typedef struct StspOp {
  int type;
  // STAGE
  int phys, dtype, bx, by;
  StageDesc stage;
  // PACK
  const void* q;
  int S, F;
  const int* idx;
  int ns;
  void* send;
  // COMM_START: one grouped ncclSend/ncclRecv per peer on the comm stream
  int npeers;
  int send_peer[STSP_MAX_PEERS], send_off[STSP_MAX_PEERS], send_cnt[STSP_MAX_PEERS];
  int nrecv;
  int recv_peer[STSP_MAX_PEERS], recv_off[STSP_MAX_PEERS], recv_cnt[STSP_MAX_PEERS];
  void* sendbuf;
  void* recvbuf;
  int slot_elems;  // elements per slot (= F)
  // FUSED: one whole SSP-RK step (fused_step.hip); the descriptor is owned by
  // the caller and must outlive the runtime (dt is rewritten by stsp_rt_set_dt).
  // MARCH3: the pipelined streaming step (march3_kernel.hip) with `stage`
  // (step input Q, output out, dt) and `fused` pointing at its March3Desc;
  // `by` = rows per segment.
  void* fused;
  // IPC copy transport (ops/native_runtime.py::IpcExchange; graph-capturable,
  // no RCCL).  IPC_SEND, in order on the compute stream (on the comm stream
  // after an event fork, joined by IPC_WAIT, with STSP_IPC_FORK=1): one
  // copy kernel (4 workgroups per send peer k) stores send_cnt[k]
  // slot_elems-element cells from sendbuf + send_off[k] into ipc_dst[k] (the
  // peer's receive slot this op fills, IPC-mapped) and releases them at
  // system scope; the last workgroup of peer k sets ipc_flag[k] (the peer's
  // flag word for this rank) = counters[0] + 1.  IPC_WAIT, on the compute stream (after the
  // join): a bounded spin until every ipc_my_flag[k] (k < nrecv) >=
  // counters[1] + 1, then counters[1] += 1 and counters[0] += 1 (the boundary
  // stage then reads the slot); a timeout sets ipc_err.  counters[4 + k] count
  // peer k's finished slices.  The counters only grow, so replayed graphs keep
  // their meaning.
  void* ipc_dst[STSP_MAX_PEERS];
  unsigned* ipc_flag[STSP_MAX_PEERS];
  unsigned* ipc_my_flag;
  unsigned* ipc_counters;
  unsigned* ipc_err;
  long long ipc_timeout_ticks;
} StspOp;

typedef struct StspRtDesc {
  int nops;
  const StspOp* ops;      // ops of `period` steps
  int period;             // steps covered by the op list
  int use_graph;          // capture graph_periods * period steps into one hipGraph
  int graph_periods;
  void* stream;           // compute stream (hipStream_t), never the legacy null stream when use_graph
  void* nccl_comm;        // ncclComm_t (nullable when there is no COMM op)
  int roctx;              // emit roctx ranges around ops (eager runs)
} StspRtDesc;

void* stsp_rt_create(const StspRtDesc* d);
void stsp_rt_destroy(void* rt);
int stsp_rt_run(void* rt, int nsteps);          // nsteps must be a multiple of period
const char* stsp_rt_last_error(void* rt);
int stsp_rt_set_dt(void* rt, double dt);         // rewrites dt in every stage op; drops the graph

int stsp_nccl_id_bytes(void);
int stsp_nccl_unique_id(void* out);              // out: stsp_nccl_id_bytes() bytes
void* stsp_nccl_comm_init(int nranks, const void* id, int rank, int device);
int stsp_nccl_comm_destroy(void* comm);
int stsp_nccl_selftest(void* comm, void* stream);   // 1-element send/recv to self (rank-local check)

int stsp_roctx_push(const char* msg);
int stsp_roctx_pop(void);
}
