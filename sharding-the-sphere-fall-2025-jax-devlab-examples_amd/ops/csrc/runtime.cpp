// Native step runtime for the cubed-sphere solver (see runtime.h).
//
// One rank's time step is a fixed op list (built once in Python from the
// integrator and the halo plan):
//
//   per RK stage, same-rank only :  STAGE(all blocks)
//   per RK stage, with remote peers:
//       PACK (compute stream)            boundary cells -> send buffer
//       COMM_START                       event: compute -> comm stream, then ONE
//                                        ncclGroupStart/End with a send and a recv
//                                        per peer (bundled fields/layers/tiles)
//       STAGE(interior blocks)           overlaps the transfer
//       COMM_WAIT                        event: comm -> compute stream
//       STAGE(boundary blocks)           remote ghosts from the receive buffer
//   per step, fused (one rank, SSP-RK3 PLR shallow water):
//       FUSED                            the whole step in one launch (fused_step.hip)
//
// The list is executed eagerly or captured once into a hipGraph (several steps
// per graph) and replayed, which removes host launch overhead entirely
// (SURVEY.md 7.1 "Step capture").  The comm stream has the highest priority
// so halo traffic is never queued behind interior work.
#include "runtime.h"

#include "rccl_abi.h"

#include <dlfcn.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

// ---- RCCL, resolved at run time (rccl_abi.h) -------------------------------------

namespace {
RcclApi g_rccl{};
std::string g_rccl_err;
bool g_rccl_done = false;

template <typename F>
bool rccl_sym(void* h, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(h, name));
  if (!out) g_rccl_err = std::string("librccl.so.1 has no ") + name;
  return out != nullptr;
}
}  // namespace

const RcclApi* rccl_api() {
  if (g_rccl_done) return g_rccl.version ? &g_rccl : nullptr;
  g_rccl_done = true;
  // STSP_RCCL_LIB=<path>: that RCCL (e.g. ROCm's /opt/rocm/lib/librccl.so.1.0.70200)
  // beside PyTorch's copy, its own symbols bound first (RTLD_DEEPBIND, local);
  // its HIP runtime dependency resolves to the one already loaded (same
  // soname), so torch streams stay usable.  Else the copy already in the
  // process (PyTorch's), else the one on the search path.
  void* h = nullptr;
  static std::string alt_path;
  if (const char* alt = std::getenv("STSP_RCCL_LIB")) {
    h = dlopen(alt, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
    if (!h) {
      g_rccl_err = std::string("cannot load STSP_RCCL_LIB=") + alt + ": " + dlerror();
      return nullptr;
    }
    alt_path = std::string(alt) + " (STSP_RCCL_LIB, deepbind)";
    g_rccl.path = alt_path.c_str();
  }
  if (!h) {
    h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    g_rccl.path = "librccl.so.1 (already loaded)";
  }
  if (!h) {
    h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    g_rccl.path = "librccl.so.1 (dlopen)";
  }
  if (!h) {
    g_rccl_err = std::string("cannot load librccl.so.1: ") + dlerror();
    return nullptr;
  }
  RcclApi a{};
  a.path = g_rccl.path;
  if (!rccl_sym(h, "ncclGetVersion", a.GetVersion) || !rccl_sym(h, "ncclGetUniqueId", a.GetUniqueId) ||
      !rccl_sym(h, "ncclCommInitRank", a.CommInitRank) || !rccl_sym(h, "ncclCommDestroy", a.CommDestroy) ||
      !rccl_sym(h, "ncclCommUserRank", a.CommUserRank) || !rccl_sym(h, "ncclSend", a.Send) ||
      !rccl_sym(h, "ncclRecv", a.Recv) || !rccl_sym(h, "ncclGroupStart", a.GroupStart) ||
      !rccl_sym(h, "ncclGroupEnd", a.GroupEnd) || !rccl_sym(h, "ncclGetErrorString", a.GetErrorString))
    return nullptr;
  int v = 0;
  if (a.GetVersion(&v) != ncclSuccess || v <= 0) {
    g_rccl_err = "ncclGetVersion failed";
    return nullptr;
  }
  if (v < STSP_RCCL_MIN_VERSION || v > STSP_RCCL_MAX_VERSION) {
    g_rccl_err = "loaded RCCL version " + std::to_string(v) + " is outside the API range this runtime declares [" +
                 std::to_string(STSP_RCCL_MIN_VERSION) + ", " + std::to_string(STSP_RCCL_MAX_VERSION) + "]";
    return nullptr;
  }
  a.version = v;
  g_rccl = a;
  return &g_rccl;
}

// Host wait mode of a device: spin (hipDeviceScheduleSpin) instead of the
// runtime's default, so a synchronize returns as soon as the GPU is done
// rather than after a yield / interrupt wake-up.  Call before the device's
// context is created (the first HIP call on it); returns the hipError_t.
extern "C" int stsp_schedule_spin(int device) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  return (int)hipSetDeviceFlags(hipDeviceScheduleSpin);
}

extern "C" int stsp_device_flags(void) {
  unsigned f = 0;
  return hipGetDeviceFlags(&f) == hipSuccess ? (int)f : -1;
}

// sizes of the C ABI descriptors, checked against the ctypes mirrors (ops/native.py)
extern "C" int stsp_desc_size(int which) {
  return which == 0 ? (int)sizeof(StageDesc) : which == 1 ? (int)sizeof(FusedDesc)
       : which == 2 ? (int)sizeof(StspOp) : which == 3 ? (int)sizeof(March3Desc) : -1;
}

extern "C" int stsp_rccl_version(void) {
  const RcclApi* r = rccl_api();
  return r ? r->version : -1;
}

extern "C" const char* stsp_rccl_error(void) { return g_rccl_err.c_str(); }

// which librccl the runtime resolved (after stsp_rccl_version() succeeded)
extern "C" const char* stsp_rccl_path(void) {
  const RcclApi* r = rccl_api();
  return r && r->path ? r->path : "";
}

namespace {

struct Runtime {
  std::vector<StspOp> ops;
  int period = 1;
  bool use_graph = false;
  int graph_periods = 1;
  hipStream_t stream = nullptr;
  hipStream_t comm_stream = nullptr;
  ncclComm_t comm = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  bool roctx = false;
  bool warmed = false;   // one eager period has run (RCCL/stream lazy setup done)
  std::string err;
};

#define RT_CHECK(expr)                                                                     \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) {                                                                \
      rt->err = std::string(#expr) + ": " + hipGetErrorString(e_);                         \
      return -1;                                                                           \
    }                                                                                      \
  } while (0)

#define NC_CHECK(expr)                                                                     \
  do {                                                                                     \
    ncclResult_t r_ = (expr);                                                              \
    if (r_ != ncclSuccess) {                                                               \
      rt->err = std::string(#expr) + ": " + rccl_api()->GetErrorString(r_);                \
      return -2;                                                                           \
    }                                                                                      \
  } while (0)

bool ipc_fork() {
  static const bool f = [] {
    const char* e = getenv("STSP_IPC_FORK");
    return e && e[0] == '1';
  }();
  return f;
}

ncclDataType_t nccl_type(int dtype) { return dtype == 1 ? ncclFloat64 : ncclFloat32; }

// IPC copy transport: the copies and signals of one exchange, and its wait
// (StspOp docs).  counters[0]: exchanges this rank has sent, counters[1]:
// exchanges it has received (both advanced by the wait kernel, which runs
// after the copy kernel has finished), counters[4 + k]: slices of peer k
// copied so far (monotonic).
struct IpcCopy {
  const char* src[STSP_MAX_PEERS];
  char* dst[STSP_MAX_PEERS];
  unsigned long long bytes[STSP_MAX_PEERS];
  unsigned* flag[STSP_MAX_PEERS];
};
constexpr int IPC_SLICES = 4;        // workgroups per peer
typedef __attribute__((address_space(1))) unsigned rt_gu32;
typedef __attribute__((address_space(1))) unsigned long long rt_gu64;
// One kernel per exchange instead of a hipMemcpyAsync per peer and a signal
// kernel (each copy node cost ~30 us per stage, profiles/r5_rehearse).  Slice
// sl of peer k is copied in V-sized words, four loads in flight per thread;
// every wave drains its stores, workgroup 0-thread releases them to system
// scope (L2 write-back), and the last slice of a peer to finish (told by a
// monotonic per-peer counter) stores the peer's flag.
template <typename V>
__global__ void __launch_bounds__(256) ipc_copy_signal_kernel(unsigned* counters, IpcCopy c) {
  const int k = blockIdx.x / IPC_SLICES, sl = blockIdx.x % IPC_SLICES;
  const unsigned long long n = c.bytes[k] / sizeof(V);   // host checked: a multiple of sizeof(V), aligned
  const unsigned long long per = (n + IPC_SLICES - 1) / IPC_SLICES;
  const unsigned long long b0 = per * sl, b1 = b0 + per < n ? b0 + per : n;
  const V* src = reinterpret_cast<const V*>(c.src[k]);
  V* dst = reinterpret_cast<V*>(c.dst[k]);
  constexpr unsigned U = 4;
  unsigned long long i = b0 + threadIdx.x;
  for (; i + (U - 1) * 256 < b1; i += U * 256) {
    V r[U];
#pragma unroll
    for (unsigned u = 0; u < U; ++u) r[u] = src[i + u * 256];
#pragma unroll
    for (unsigned u = 0; u < U; ++u) dst[i + u * 256] = r[u];
  }
  for (; i < b1; i += 256) dst[i] = src[i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);                // system scope: write back L2
    const unsigned done = __hip_atomic_fetch_add((rt_gu32*)(counters + 4 + k), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (done % IPC_SLICES == 0) {
      __atomic_thread_fence(__ATOMIC_SEQ_CST);
      __hip_atomic_store((rt_gu32*)c.flag[k], counters[0] + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
__global__ void ipc_wait_kernel(unsigned* counters, const unsigned* my, int n, unsigned* err, long long ticks) {
  __shared__ unsigned want;
  if (threadIdx.x == 0) want = counters[1] + 1u;
  __syncthreads();
  const int k = threadIdx.x;
  if (k < n) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load((rt_gu32*)(my + k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
      if (__hip_atomic_load((rt_gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > ticks) {
        __hip_atomic_store((rt_gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    counters[1] = want;
    counters[0] += 1u;                 // this rank's copy kernel of the exchange has finished (join)
  }
}
size_t elem_bytes(int dtype) { return dtype == 1 ? 8 : 4; }

int run_op(Runtime* rt, const StspOp& op) {
  switch (op.type) {
    case STSP_OP_STAGE: {
      const int rc = stsp_stage_launch(op.phys, op.dtype, op.bx, op.by, &op.stage, rt->stream);
      if (rc != 0) {
        rt->err = "stage launch failed: " + std::to_string(rc);
        return -3;
      }
      return 0;
    }
    case STSP_OP_PACK: {
      const int rc = stsp_pack_launch(op.dtype, op.q, op.S, op.F, op.idx, op.ns, op.send, rt->stream);
      if (rc != 0) {
        rt->err = "pack launch failed: " + std::to_string(rc);
        return -3;
      }
      return 0;
    }
    case STSP_OP_COMM_START: {
      if (!rt->comm) {
        rt->err = "COMM op without an RCCL communicator";
        return -4;
      }
      RT_CHECK(hipEventRecord(rt->ev_fork, rt->stream));
      RT_CHECK(hipStreamWaitEvent(rt->comm_stream, rt->ev_fork, 0));
      const size_t eb = elem_bytes(op.dtype);
      const ncclDataType_t ty = nccl_type(op.dtype);
      const RcclApi* R = rccl_api();       // non-null: the communicator was made through it
      NC_CHECK(R->GroupStart());
      for (int k = 0; k < op.npeers; ++k) {
        const char* p = static_cast<const char*>(op.sendbuf) + (size_t)op.send_off[k] * op.slot_elems * eb;
        NC_CHECK(R->Send(p, (size_t)op.send_cnt[k] * op.slot_elems, ty, op.send_peer[k], rt->comm, rt->comm_stream));
      }
      for (int k = 0; k < op.nrecv; ++k) {
        char* p = static_cast<char*>(op.recvbuf) + (size_t)op.recv_off[k] * op.slot_elems * eb;
        NC_CHECK(R->Recv(p, (size_t)op.recv_cnt[k] * op.slot_elems, ty, op.recv_peer[k], rt->comm, rt->comm_stream));
      }
      NC_CHECK(R->GroupEnd());
      return 0;
    }
    case STSP_OP_FUSED: {
      const int rc = stsp_fused_launch(op.dtype, static_cast<const FusedDesc*>(op.fused), rt->stream);
      if (rc != 0) {
        rt->err = "fused step launch failed: " + std::to_string(rc);
        return -3;
      }
      return 0;
    }
    case STSP_OP_MARCH3: {
      const int rc = stsp_march3_launch(op.dtype, op.by, &op.stage, static_cast<const March3Desc*>(op.fused),
                                        rt->stream);
      if (rc != 0) {
        rt->err = "pipelined march launch failed: " + std::to_string(rc);
        return -3;
      }
      return 0;
    }
    case STSP_OP_COMM_WAIT: {
      RT_CHECK(hipEventRecord(rt->ev_join, rt->comm_stream));
      RT_CHECK(hipStreamWaitEvent(rt->stream, rt->ev_join, 0));
      return 0;
    }
    case STSP_OP_IPC_SEND: {
      if (!op.ipc_counters || op.npeers > STSP_MAX_PEERS) {
        rt->err = "IPC_SEND op without counters";
        return -4;
      }
      // STSP_IPC_FORK=1: the copy kernel runs on the comm stream, overlapping
      // the interior stage; default: in order on the compute stream (the
      // cross-stream fork and join of a graph cost more than the copy).
      const bool fork = ipc_fork();
      hipStream_t cs = fork ? rt->comm_stream : rt->stream;
      if (fork) {
        RT_CHECK(hipEventRecord(rt->ev_fork, rt->stream));
        RT_CHECK(hipStreamWaitEvent(rt->comm_stream, rt->ev_fork, 0));
      }
      const size_t eb = elem_bytes(op.dtype);
      IpcCopy cp;
      for (int k = 0; k < op.npeers; ++k) {
        cp.src[k] = static_cast<const char*>(op.sendbuf) + (size_t)op.send_off[k] * op.slot_elems * eb;
        cp.dst[k] = static_cast<char*>(op.ipc_dst[k]);
        cp.bytes[k] = (unsigned long long)op.send_cnt[k] * op.slot_elems * eb;
        cp.flag[k] = op.ipc_flag[k];
      }
      if (op.npeers > 0) {
        bool w16 = true;                 // 16-byte words when every pointer and size allows
        for (int k = 0; k < op.npeers; ++k)
          w16 = w16 && (((uintptr_t)cp.src[k] | (uintptr_t)cp.dst[k] | (uintptr_t)cp.bytes[k]) % 16 == 0);
        bool w4 = true;
        for (int k = 0; k < op.npeers; ++k)
          w4 = w4 && (((uintptr_t)cp.src[k] | (uintptr_t)cp.dst[k] | (uintptr_t)cp.bytes[k]) % 4 == 0);
        if (!w4) {
          rt->err = "IPC_SEND: payloads must be 4-byte aligned";
          return -1;
        }
        if (w16)
          hipLaunchKernelGGL(ipc_copy_signal_kernel<uint4>, dim3(op.npeers * IPC_SLICES), dim3(256), 0,
                             cs, op.ipc_counters, cp);
        else
          hipLaunchKernelGGL(ipc_copy_signal_kernel<unsigned>, dim3(op.npeers * IPC_SLICES), dim3(256), 0,
                             cs, op.ipc_counters, cp);
        RT_CHECK(hipGetLastError());
      }
      // joined by the IPC_WAIT after the interior stage (the copies overlap it;
      // the next PACK, which overwrites sendbuf, comes after that join)
      if (fork) RT_CHECK(hipEventRecord(rt->ev_join, rt->comm_stream));
      return 0;
    }
    case STSP_OP_IPC_WAIT: {
      if (!op.ipc_counters || !op.ipc_my_flag || !op.ipc_err || op.nrecv > 64) {
        rt->err = "IPC_WAIT op without flags";
        return -4;
      }
      if (ipc_fork()) RT_CHECK(hipStreamWaitEvent(rt->stream, rt->ev_join, 0));   // this rank's copies are out
      hipLaunchKernelGGL(ipc_wait_kernel, dim3(1), dim3(64), 0, rt->stream, op.ipc_counters, op.ipc_my_flag,
                         op.nrecv, op.ipc_err, op.ipc_timeout_ticks);
      RT_CHECK(hipGetLastError());
      return 0;
    }
  }
  rt->err = "unknown op type " + std::to_string(op.type);
  return -5;
}

bool debug_enabled() {
  static const bool on = [] {
    const char* v = std::getenv("STSP_RT_DEBUG");
    return v && v[0] == '1';
  }();
  return on;
}

int run_period(Runtime* rt, bool mark) {
  for (const StspOp& op : rt->ops) {
    if (debug_enabled()) {
      std::fprintf(stderr, "[stsp_rt] op type=%d phys=%d nblocks=%d remote=%d npeers=%d nrecv=%d comm=%p\n", op.type,
                   op.phys, op.stage.nblocks, op.stage.remote, op.npeers, op.nrecv, (void*)rt->comm);
      std::fflush(stderr);
    }
    if (mark) {
      const char* names[] = {"?", "stage", "pack", "comm", "comm_wait", "fused_step", "ipc_send", "ipc_wait"};
      roctxRangePush(names[op.type >= 1 && op.type <= 7 ? op.type : 0]);
    }
    const int rc = run_op(rt, op);
    if (mark) roctxRangePop();
    if (rc) return rc;
  }
  return 0;
}

int graph_mode() {
  static const int m = [] {
    const char* v = std::getenv("STSP_GRAPH_MODE");
    return v ? std::atoi(v) : 0;
  }();
  return m;
}

int ensure_graph(Runtime* rt) {
  if (rt->exec) return 0;
  const int gm = graph_mode();
  RT_CHECK(hipStreamBeginCapture(rt->stream, (gm & 1) ? hipStreamCaptureModeGlobal : hipStreamCaptureModeRelaxed));
  int rc = 0;
  for (int p = 0; p < rt->graph_periods && rc == 0; ++p) rc = run_period(rt, false);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(rt->stream, &g);
  if (rc) {
    if (g) hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) {
    rt->err = std::string("hipStreamEndCapture: ") + hipGetErrorString(e);
    return -1;
  }
  rt->graph = g;
  if (gm & 2) {
    const char* fv = std::getenv("STSP_GRAPH_IFLAGS");
    RT_CHECK(hipGraphInstantiateWithFlags(&rt->exec, rt->graph, fv ? std::strtoull(fv, nullptr, 0) : 0));
  }
  else
    RT_CHECK(hipGraphInstantiate(&rt->exec, rt->graph, nullptr, nullptr, 0));
  if (gm & 4) RT_CHECK(hipGraphUpload(rt->exec, rt->stream));
  return 0;
}

void drop_graph(Runtime* rt) {
  if (rt->exec) hipGraphExecDestroy(rt->exec);
  if (rt->graph) hipGraphDestroy(rt->graph);
  rt->exec = nullptr;
  rt->graph = nullptr;
}

}  // namespace

extern "C" void* stsp_rt_create(const StspRtDesc* d) {
  auto* rt = new Runtime();
  if (debug_enabled())
    std::fprintf(stderr, "[stsp_rt] create nops=%d period=%d graph=%d sizeof(StspOp)=%zu sizeof(StageDesc)=%zu\n",
                 d->nops, d->period, d->use_graph, sizeof(StspOp), sizeof(StageDesc));
  rt->ops.assign(d->ops, d->ops + d->nops);
  rt->period = d->period > 0 ? d->period : 1;
  rt->use_graph = d->use_graph != 0;
  rt->graph_periods = d->graph_periods > 0 ? d->graph_periods : 1;
  rt->stream = static_cast<hipStream_t>(d->stream);
  rt->comm = static_cast<ncclComm_t>(d->nccl_comm);
  rt->roctx = d->roctx != 0;
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  if (hipStreamCreateWithPriority(&rt->comm_stream, hipStreamNonBlocking, hi) != hipSuccess ||
      hipEventCreateWithFlags(&rt->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&rt->ev_join, hipEventDisableTiming) != hipSuccess) {
    rt->err = "stream/event creation failed";
  }
  return rt;
}

extern "C" void stsp_rt_destroy(void* p) {
  auto* rt = static_cast<Runtime*>(p);
  if (!rt) return;
  drop_graph(rt);
  if (rt->ev_fork) hipEventDestroy(rt->ev_fork);
  if (rt->ev_join) hipEventDestroy(rt->ev_join);
  if (rt->comm_stream) hipStreamDestroy(rt->comm_stream);
  delete rt;
}

extern "C" const char* stsp_rt_last_error(void* p) {
  return static_cast<Runtime*>(p)->err.c_str();
}

extern "C" int stsp_rt_set_dt(void* p, double dt) {
  auto* rt = static_cast<Runtime*>(p);
  for (StspOp& op : rt->ops) {
    if (op.type == STSP_OP_STAGE || op.type == STSP_OP_MARCH3) op.stage.dt = dt;
    if (op.type == STSP_OP_FUSED && op.fused) static_cast<FusedDesc*>(op.fused)->dt = dt;
  }
  drop_graph(rt);
  return 0;
}

extern "C" int stsp_rt_run(void* p, int nsteps) {
  auto* rt = static_cast<Runtime*>(p);
  if (!rt->err.empty() && !rt->comm_stream) return -6;
  if (nsteps % rt->period) {
    rt->err = "nsteps must be a multiple of the op-list period";
    return -7;
  }
  int periods = nsteps / rt->period;
  if (rt->use_graph && !rt->warmed && periods > 0) {
    // RCCL and the comm stream do lazy one-time setup on first use, which is
    // illegal inside a capture: run the first period eagerly (it counts).
    const int rc = run_period(rt, rt->roctx);
    if (rc) return rc;
    RT_CHECK(hipStreamSynchronize(rt->stream));
    rt->warmed = true;
    --periods;
  }
  if (rt->use_graph && periods >= rt->graph_periods) {
    const int rc = ensure_graph(rt);
    if (rc) return rc;
    const int launches = periods / rt->graph_periods;
    hipStream_t ls = (graph_mode() & 8) ? nullptr : rt->stream;
    if (ls != rt->stream) {
      RT_CHECK(hipEventRecord(rt->ev_fork, rt->stream));
      RT_CHECK(hipStreamWaitEvent(ls, rt->ev_fork, 0));
    }
    for (int i = 0; i < launches; ++i) RT_CHECK(hipGraphLaunch(rt->exec, ls));
    if (ls != rt->stream) {
      RT_CHECK(hipEventRecord(rt->ev_join, ls));
      RT_CHECK(hipStreamWaitEvent(rt->stream, rt->ev_join, 0));
    }
    periods -= launches * rt->graph_periods;
  }
  for (int i = 0; i < periods; ++i) {
    const int rc = run_period(rt, rt->roctx);
    if (rc) return rc;
  }
  return 0;
}

// ---- RCCL bootstrap -----------------------------------------------------------

extern "C" int stsp_nccl_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

extern "C" int stsp_nccl_unique_id(void* out) {
  const RcclApi* R = rccl_api();
  if (!R) return -2;
  ncclUniqueId id;
  if (R->GetUniqueId(&id) != ncclSuccess) return -1;
  std::memcpy(out, &id, sizeof(id));
  return 0;
}

extern "C" void* stsp_nccl_comm_init(int nranks, const void* idbytes, int rank, int device) {
  const RcclApi* R = rccl_api();
  if (!R) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  ncclUniqueId id;
  std::memcpy(&id, idbytes, sizeof(id));
  ncclComm_t comm = nullptr;
  const ncclResult_t r = R->CommInitRank(&comm, nranks, id, rank);
  if (r != ncclSuccess) {
    g_rccl_err = std::string("ncclCommInitRank: ") + R->GetErrorString(r);
    return nullptr;
  }
  return comm;
}

extern "C" int stsp_nccl_comm_destroy(void* comm) {
  if (!comm) return 0;
  const RcclApi* R = rccl_api();
  return R && R->CommDestroy(static_cast<ncclComm_t>(comm)) == ncclSuccess ? 0 : -1;
}

extern "C" int stsp_nccl_selftest(void* comm, void* stream) {
  // 1-element send/recv to self through the same grouped path the halo uses.
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  const RcclApi* R = rccl_api();
  if (!R) return -5;
  int rank = 0;
  if (R->CommUserRank(c, &rank) != ncclSuccess) return -1;
  double* buf = nullptr;
  if (hipMalloc(&buf, 2 * sizeof(double)) != hipSuccess) return -2;
  const double v = 42.0 + rank;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipMemcpyAsync(buf, &v, sizeof(double), hipMemcpyHostToDevice, s);
  hipMemsetAsync(buf + 1, 0, sizeof(double), s);
  R->GroupStart();
  R->Send(buf, 1, ncclFloat64, rank, c, s);
  R->Recv(buf + 1, 1, ncclFloat64, rank, c, s);
  const ncclResult_t r = R->GroupEnd();
  double out = 0;
  hipMemcpyAsync(&out, buf + 1, sizeof(double), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  hipFree(buf);
  if (r != ncclSuccess) return -3;
  return out == v ? 0 : -4;
}

// ---- direct xGMI halo memory (ops/xgmi.py) -------------------------------------
// One uncached device allocation per rank holds its arrival counters and its
// receive ring; peers map it through a dmabuf IPC handle and store into it
// over xGMI.  Uncached (MTYPE UC) so neither the owner's nor a peer's L2 keeps
// a line of it; every kernel access is additionally system scope.

// Ring memory stays with the process once allocated: a freed ring goes on a
// free list and the next ring that fits reuses it (zeroed).  Handing uncached
// memory back with hipFree was followed by corrupted values in ordinary
// allocations made afterwards (a test after the loopback test read NaN and
// garbage from fresh torch buffers in 5 of 6 runs; never with the ring kept,
// profiles/r4_ring/README.md), and a ring peers have mapped should not
// return to the driver under them anyway.
//
// Diagnostics (STSP_RING_GUARD=1): every ring gets a guard region of
// RING_GUARD bytes on each side, filled with a pattern at allocation and
// checked by stsp_xg_check_guards() (the GPU tests call it after every test
// in that mode): a kernel store past either end of a ring shows up there.
// STSP_XG_POOL=0 hands rings back with hipFree again (the experiment of
// profiles/r4_ring, kept for re-runs).
namespace {
std::mutex g_ring_mu;
std::unordered_map<void*, size_t> g_ring_bytes;   // every ring ever allocated
std::vector<void*> g_ring_free;                   // of those, the free ones
constexpr size_t RING_GUARD = 65536;
constexpr unsigned GUARD_WORD = 0x5A17C0DEu;
bool env_on(const char* name, bool dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) != 0 : dflt;
}
bool ring_guard() {
  static const bool on = env_on("STSP_RING_GUARD", false);
  return on;
}
bool ring_pool() {
  static const bool on = env_on("STSP_XG_POOL", true);
  return on;
}
__global__ void guard_fill_kernel(unsigned* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = GUARD_WORD;
}
__global__ void guard_check_kernel(const unsigned* p, size_t n, unsigned* bad) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    if (p[i] != GUARD_WORD) atomicAdd(bad, 1u);
}
}  // namespace

extern "C" int stsp_xg_alloc(size_t bytes, void** out) {
  *out = nullptr;
  void* p = nullptr;
  size_t have = 0;
  if (ring_pool()) {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    size_t best = 0;
    for (size_t k = 0; k < g_ring_free.size(); ++k) {   // smallest free ring that fits
      const size_t b = g_ring_bytes[g_ring_free[k]];
      if (b >= bytes && (!p || b < have)) { p = g_ring_free[k]; have = b; best = k; }
    }
    if (p) g_ring_free.erase(g_ring_free.begin() + best);
  }
  if (!p) {
    const size_t g = ring_guard() ? RING_GUARD : 0;
    void* raw = nullptr;
    if (hipExtMallocWithFlags(&raw, bytes + 2 * g, hipDeviceMallocUncached) != hipSuccess) return -1;
    if (g) {
      hipLaunchKernelGGL(guard_fill_kernel, dim3(64), dim3(256), 0, 0, (unsigned*)raw, g / 4);
      hipLaunchKernelGGL(guard_fill_kernel, dim3(64), dim3(256), 0, 0, (unsigned*)((char*)raw + g + bytes), g / 4);
    }
    p = (char*)raw + g;
    have = bytes;
    std::lock_guard<std::mutex> lk(g_ring_mu);
    g_ring_bytes[p] = bytes;
  }
  if (hipMemset(p, 0, have) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    g_ring_free.push_back(p);
    return -2;
  }
  *out = p;
  return 0;
}

// Guard words of every ring this process holds that differ from the pattern
// (STSP_RING_GUARD=1; 0 otherwise or when clean, < 0 on a HIP error).
extern "C" long long stsp_xg_check_guards(void) {
  if (!ring_guard()) return 0;
  std::vector<void*> rings;
  std::vector<size_t> sizes;
  {
    std::lock_guard<std::mutex> lk(g_ring_mu);
    for (auto& kv : g_ring_bytes) { rings.push_back(kv.first); sizes.push_back(kv.second); }
  }
  unsigned* d = nullptr;
  if (hipMalloc(&d, sizeof(unsigned)) != hipSuccess) return -1;
  hipMemset(d, 0, sizeof(unsigned));
  for (size_t k = 0; k < rings.size(); ++k) {
    char* p = (char*)rings[k];
    hipLaunchKernelGGL(guard_check_kernel, dim3(64), dim3(256), 0, 0, (const unsigned*)(p - RING_GUARD),
                       RING_GUARD / 4, d);
    hipLaunchKernelGGL(guard_check_kernel, dim3(64), dim3(256), 0, 0, (const unsigned*)(p + sizes[k]),
                       RING_GUARD / 4, d);
  }
  unsigned h = 0;
  const bool ok = hipMemcpy(&h, d, sizeof(unsigned), hipMemcpyDeviceToHost) == hipSuccess;
  hipFree(d);
  return ok ? (long long)h : -2;
}

// Ordinary device memory for IPC payload slots (zeroed), and its release.
extern "C" int stsp_dev_alloc(size_t bytes, void** out) {
  *out = nullptr;
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return -1;
  if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    hipFree(p);
    return -2;
  }
  *out = p;
  return 0;
}

extern "C" int stsp_dev_free(void* p) {
  if (!p) return 0;
  if (hipDeviceSynchronize() != hipSuccess) return -2;
  return hipFree(p) == hipSuccess ? 0 : -3;
}

// Device allocation with explicit hipExtMallocWithFlags flags (zeroed):
// 1 = fine-grained, 3 = uncached (exchange-buffer memory-type experiments).
extern "C" int stsp_alloc_flags(size_t bytes, unsigned flags, void** out) {
  *out = nullptr;
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, flags) != hipSuccess) return -1;
  if (hipMemset(p, 0, bytes) != hipSuccess) {
    hipFree(p);
    return -2;
  }
  if (hipDeviceSynchronize() != hipSuccess) return -3;
  *out = p;
  return 0;
}

extern "C" int stsp_xg_free(void* p) {
  if (!p) return 0;
  std::lock_guard<std::mutex> lk(g_ring_mu);
  if (!g_ring_bytes.count(p)) return -1;   // not a ring of this process
  for (void* q : g_ring_free)
    if (q == p) return -1;                 // freed twice
  if (!ring_pool()) {                      // STSP_XG_POOL=0: back to the driver (diagnostics)
    if (hipDeviceSynchronize() != hipSuccess) return -2;
    const size_t g = ring_guard() ? RING_GUARD : 0;
    g_ring_bytes.erase(p);
    return hipFree((char*)p - g) == hipSuccess ? 0 : -3;
  }
  g_ring_free.push_back(p);
  return 0;
}

// Rings held by the process (allocated, free) and their bytes.
extern "C" int stsp_xg_pool(long long* out4) {
  std::lock_guard<std::mutex> lk(g_ring_mu);
  long long tot = 0, fb = 0;
  for (auto& kv : g_ring_bytes) tot += (long long)kv.second;
  for (void* q : g_ring_free) fb += (long long)g_ring_bytes[q];
  out4[0] = (long long)g_ring_bytes.size();
  out4[1] = (long long)g_ring_free.size();
  out4[2] = tot;
  out4[3] = fb;
  return 0;
}

extern "C" int stsp_ipc_handle_bytes(void) { return HIP_IPC_HANDLE_SIZE; }

extern "C" int stsp_ipc_get(void* p, void* handle_out) {
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, p);
  if (e != hipSuccess) return (int)e;
  std::memcpy(handle_out, &h, sizeof(h));
  return 0;
}

extern "C" int stsp_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  *out = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
  return e == hipSuccess ? 0 : (int)e;
}

// Offset of p inside its allocation (an IPC mapping opens at the allocation's
// base: a ring behind a guard region, STSP_RING_GUARD=1, starts past it).
extern "C" long long stsp_ipc_offset(void* p) {
  hipDeviceptr_t base = nullptr;
  size_t sz = 0;
  if (hipMemGetAddressRange(&base, &sz, (hipDeviceptr_t)p) != hipSuccess) return -1;
  return (long long)((char*)p - (char*)base);
}

extern "C" int stsp_ipc_close(void* p) { return hipIpcCloseMemHandle(p) == hipSuccess ? 0 : -1; }

// Best effort: map every other visible GPU for peer access (already-enabled and
// not-possible are not errors here; IPC mappings carry their own access).
extern "C" int stsp_enable_peers(int device) {
  int n = 0, ok = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -1;
  for (int p = 0; p < n; ++p) {
    if (p == device) continue;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, device, p) == hipSuccess && can) {
      const hipError_t e = hipDeviceEnablePeerAccess(p, 0);
      if (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled) ++ok;
      else (void)hipGetLastError();
    }
  }
  return ok;
}

extern "C" int stsp_roctx_push(const char* msg) { return roctxRangePush(msg); }
extern "C" int stsp_roctx_pop(void) { return roctxRangePop(); }
