// SPDX-License-Identifier: MIT
// Link probe: what this node's GPU-to-GPU paths deliver, measured by the ranks themselves before
// the data-path tuner times any candidate (grayscott_amd/parallel/linkprobe.py, bench.py
// "link_probe"; parallel/autotune.py prunes with the result).
//
// The reference has one exchange and never measures it (communication.jl:138-199: blocking
// MPI.Sendrecv! of host-staged faces).  Here the tuner chooses between z slabs (two neighbours,
// whole planes: 6.3 MB per message for a 512^2 fp32 plane pair at T = 3) and the 2x2x2 grid (up to
// seven neighbours, 1.5 MB faces over separate links), over RCCL or the IPC peer-store transport,
// and which one wins depends on the per-link rate at THOSE sizes -- xGMI is point to point, so a
// rank's exchange is bound by its slowest neighbour link, not by a switch.  Each pair of ranks
// therefore measures, both directions at once (as a halo exchange runs):
//   * IPC peer stores: a copy kernel storing 16 B per lane from local HBM straight into the
//     peer's uncached buffer (the same store path as the IPC transport's pack kernel), at the
//     message sizes the candidates send, plus the time of a 4 KB put (launch + link latency);
//   * RCCL point-to-point: one ncclGroup of send + recv with the partner at the same sizes, on a
//     communicator set up non-blocking and polled under GS_COMM_TIMEOUT.  A communicator made
//     here is handed to the engines (SharedComm), so the bootstrap is paid once.
// Every probe call is synchronous and bounded: a put kernel moves a fixed byte count, and an RCCL
// group that does not finish within GS_COMM_TIMEOUT aborts the communicator and raises.
#pragma once

#include <map>
#include <string>
#include <vector>

namespace {

// grid-stride 16-byte copy src -> dst (dst: a peer's buffer mapped through IPC)
__global__ __launch_bounds__(256) void k_probe_put(const uint4* __restrict__ src,
                                                   uint4* __restrict__ dst, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

struct LinkProbe {
  int dev = 0;
  int64_t cap = 0;  // bytes of each buffer
  char* src = nullptr;
  char* dst = nullptr;   // exported (uncached, like the IPC transport's landing buffers)
  char* rbuf = nullptr;  // RCCL receive buffer
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::map<std::string, char*> peers;  // export bytes -> mapped peer buffer
  ncclComm_t comm = nullptr;
  bool comm_owned = false;  // false: the process-wide SharedComm (engines reuse it)

  explicit LinkProbe(int64_t bytes) : cap(bytes) {
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipMalloc((void**)&src, cap));
    HIP_CHECK(hipMalloc((void**)&rbuf, cap));
    HIP_CHECK(hipExtMallocWithFlags((void**)&dst, cap, hipDeviceMallocUncached));
    HIP_CHECK(hipMemset(src, 0x5a, cap));
    HIP_CHECK(hipMemset(dst, 0, cap));
    HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreate(&e0));
    HIP_CHECK(hipEventCreate(&e1));
    HIP_CHECK(hipDeviceSynchronize());
  }
  ~LinkProbe() {
    // (teardown: errors are ignored, the handles are gone either way)
    (void)hipDeviceSynchronize();
    for (auto& kv : peers) (void)hipIpcCloseMemHandle(kv.second);
    if (comm && comm_owned) ncclCommDestroy(comm);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(st);
    (void)hipFree(src);
    (void)hipFree(rbuf);
    (void)hipFree(dst);
  }

  // out: the dst buffer's IPC handle, then this device's PCI bus id
  void export_to(char* out) const {
    hipIpcMemHandle_t h;
    HIP_CHECK(hipIpcGetMemHandle(&h, dst));
    memset(out, 0, kIpcHandleBytes);
    memcpy(out, &h, sizeof(h));
    HIP_CHECK(hipDeviceGetPCIBusId(out + 2 * sizeof(hipIpcMemHandle_t), kIpcPciBytes - 1, dev));
  }

  char* map_peer(const char* exp) {
    const std::string key(exp, sizeof(hipIpcMemHandle_t));
    auto it = peers.find(key);
    if (it != peers.end()) return it->second;
    char pci[kIpcPciBytes];
    memcpy(pci, exp + 2 * sizeof(hipIpcMemHandle_t), kIpcPciBytes);
    pci[kIpcPciBytes - 1] = 0;
    int pdev = -1;
    if (pci[0] && hipDeviceGetByPCIBusId(&pdev, pci) != hipSuccess) pdev = -1;
    if (pdev >= 0 && pdev != dev) {
      int can = 0;
      HIP_CHECK(hipDeviceCanAccessPeer(&can, dev, pdev));
      if (!can)
        throw std::runtime_error("link probe: device " + std::to_string(dev) +
                                 " cannot access peer device " + std::to_string(pdev));
    }
    hipIpcMemHandle_t h;
    memcpy(&h, exp, sizeof(h));
    char* p = nullptr;
    HIP_CHECK(hipIpcOpenMemHandle((void**)&p, h, hipIpcMemLazyEnablePeerAccess));
    peers[key] = p;
    return p;
  }

  // wait for event e under GS_COMM_TIMEOUT: an RCCL receive whose partner never sends would
  // otherwise block the host forever; on a timeout the communicator is aborted (which ends its
  // kernels) and the probe raises
  void wait_event(hipEvent_t e) {
    const double to = gs::comm_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    int sleep_us = 5;
    for (;;) {
      const hipError_t q = hipEventQuery(e);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) HIP_CHECK(q);
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > to) {
        drop_comm();
        throw std::runtime_error("link probe: a timed transfer did not finish within " +
                                 std::to_string(to) + " s (GS_COMM_TIMEOUT)");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
      if (sleep_us < 1000) sleep_us *= 2;
    }
  }

  // median microseconds of `reps` timed launches of `enqueue` (one warm-up launch first)
  template <class F>
  double time_us(int reps, F&& enqueue) {
    enqueue();
    HIP_CHECK(hipEventRecord(e1, st));
    wait_event(e1);
    std::vector<float> t;
    for (int i = 0; i < reps; ++i) {
      HIP_CHECK(hipEventRecord(e0, st));
      enqueue();
      HIP_CHECK(hipEventRecord(e1, st));
      wait_event(e1);
      float ms = 0.f;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return 1e3 * (double)t[t.size() / 2];
  }

  double ipc_put(const char* exp, int64_t bytes, int reps) {
    if (bytes > cap || bytes <= 0) throw std::runtime_error("link probe: size out of range");
    char* peer = map_peer(exp);
    const int64_t n16 = bytes / 16;
    const int blocks = (int)std::min<int64_t>(std::max<int64_t>((n16 + 255) / 256, 1), 512);
    return time_us(reps, [&] {
      hipLaunchKernelGGL(k_probe_put, dim3(blocks), dim3(256), 0, st, (const uint4*)src,
                         (uint4*)peer, n16);
    });
  }

  // poll a non-blocking communicator's pending operation under GS_COMM_TIMEOUT
  void complete(const char* what) {
    const double to = gs::comm_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    int sleep_us = 10;
    for (;;) {
      ncclResult_t s = ncclSuccess;
      const ncclResult_t q = ncclCommGetAsyncError(comm, &s);
      if (q != ncclSuccess) s = q;
      if (s == ncclSuccess) return;
      const double el =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (s != ncclInProgress || el > to) {
        drop_comm();
        throw std::runtime_error(std::string("link probe: RCCL ") + what +
                                 (s != ncclInProgress ? std::string(": ") + ncclGetErrorString(s)
                                                      : std::string(" timed out (GS_COMM_TIMEOUT)")));
      }
      std::this_thread::sleep_for(std::chrono::microseconds(sleep_us));
      if (sleep_us < 1000) sleep_us *= 2;
    }
  }

  void drop_comm() {
    if (!comm) return;
    if (comm == shared_comm().comm) shared_comm() = SharedComm{};
    ncclCommAbort(comm);
    comm = nullptr;
  }

  void rccl_init(const ncclUniqueId& id, int nranks, int rank) {
    SharedComm& sc = shared_comm();
    if (sc.comm && sc.nranks == nranks && sc.rank == rank) {
      comm = sc.comm;
      return;
    }
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t c = nullptr;
    const ncclResult_t r = ncclCommInitRankConfig(&c, nranks, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (c) ncclCommAbort(c);
      throw std::runtime_error(std::string("link probe: RCCL ") + ncclGetErrorString(r) +
                               " (ncclCommInitRankConfig)");
    }
    comm = c;
    complete("communicator set-up");
    if (!sc.comm) sc = SharedComm{comm, nranks, rank};  // the engines' communicator from now on
    else comm_owned = true;
  }

  double rccl_sendrecv(int peer, int64_t bytes, int reps) {
    if (!comm) throw std::runtime_error("link probe: no RCCL communicator");
    if (bytes > cap || bytes <= 0) throw std::runtime_error("link probe: size out of range");
    auto one = [&] {
      NCCL_CHECK(ncclGroupStart());
      NCCL_CHECK(ncclSend(src, (size_t)bytes, ncclUint8, peer, comm, st));
      NCCL_CHECK(ncclRecv(rbuf, (size_t)bytes, ncclUint8, peer, comm, st));
      const ncclResult_t r = ncclGroupEnd();
      if (r == ncclInProgress) complete("send / receive connection set-up");
      else if (r != ncclSuccess)
        throw std::runtime_error(std::string("link probe: RCCL ") + ncclGetErrorString(r));
    };
    // (time_us' warm-up group makes the connection, outside the timing)
    return time_us(reps, one);
  }
};

}  // namespace

extern "C" {

void* gs_probe_create(int64_t bytes) {
  try {
    return new LinkProbe(bytes);
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return nullptr;
  }
}

void gs_probe_destroy(void* p) { delete (LinkProbe*)p; }

int gs_probe_export(void* p, char* out) {
  try {
    ((LinkProbe*)p)->export_to(out);
    return kIpcHandleBytes;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

// median microseconds of a `bytes` put into the peer whose export is `peer_export`
int gs_probe_ipc(void* p, const char* peer_export, int64_t bytes, int32_t reps, double* out_us) {
  try {
    *out_us = ((LinkProbe*)p)->ipc_put(peer_export, bytes, reps);
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

int gs_probe_rccl_init(void* p, const char* uid, int32_t nranks, int32_t rank) {
  try {
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    ((LinkProbe*)p)->rccl_init(id, nranks, rank);
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

// median microseconds of one grouped send + receive of `bytes` with `peer`
int gs_probe_rccl(void* p, int32_t peer, int64_t bytes, int32_t reps, double* out_us) {
  try {
    *out_us = ((LinkProbe*)p)->rccl_sendrecv(peer, bytes, reps);
    return 0;
  } catch (const std::exception& ex) {
    g_gs_err = ex.what();
    return -1;
  }
}

}  // extern "C"
