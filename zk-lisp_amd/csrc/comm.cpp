// Multi-GPU boundary exchange over RCCL: the one collective of
// the sharded path.  Each rank proves its own segments; what the aggregation consumes on
// rank 0 -- the zl1 step proofs with their boundary fields (agg/trace.rs:155-238 reads
// state hashes, RAM grand products and ROM lanes from them) -- is gathered there with RCCL
// point-to-point transfers between the GPUs (xGMI inside a node).  The reference has no
// collective: its segments are proved in one process and handed over as a Vec<StepProof>
// (prove.rs:1018-1050, lib.rs:382-482).
//
// RCCL is opened at run time (librccl.so.1, the ROCm image's; a process that already holds
// one, e.g. torch's, shares it), so the library loads and the single-GPU path runs without it.
#include <dlfcn.h>
#include <stdio.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/zkl_hip.h"
#include "kernels.h"
#include "proof_view.h"

namespace {

// the slice of rccl.h this file uses (NCCL 2.x ABI)
typedef struct ncclComm* ncclComm_t;
typedef struct { char internal[128]; } ncclUniqueId;
typedef int ncclResult_t;
enum { ncclUint8 = 1, ncclUint64 = 5 };

struct Rccl {
  void* h = nullptr;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // ZKL_RCCL_LIB names another NCCL-ABI library: the tests' shared-memory stub
    // (tests/stub/nccl_shm_stub.cpp) drives the multi-rank branches below with several
    // processes on one GPU, which RCCL refuses (duplicate devices)
    const char* alt = getenv("ZKL_RCCL_LIB");
    if (alt && *alt) {
      fprintf(stderr, "zkl_hip: ZKL_RCCL_LIB=%s replaces librccl (test hook)\n", alt);
      r.h = dlopen(alt, RTLD_NOW | RTLD_LOCAL);
    } else {
      r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!r.h) r.h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    }
    if (!r.h) {
      const char* e = dlerror();
      r.err = std::string("RCCL not available: ") + (e ? e : "dlopen failed");
      return;
    }
    auto sym = [&](const char* n) {
      void* p = dlsym(r.h, n);
      if (!p && r.err.empty()) r.err = std::string("RCCL symbol missing: ") + n;
      return p;
    };
    r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
    r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
    r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
    r.AllGather = (decltype(r.AllGather))sym("ncclAllGather");
    r.Send = (decltype(r.Send))sym("ncclSend");
    r.Recv = (decltype(r.Recv))sym("ncclRecv");
    r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
    r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
  });
  if (!r.err.empty()) throw std::runtime_error(r.err);
  return r;
}

void nccl_check(ncclResult_t e, const char* what) {
  if (e != 0) {
    const char* s = rccl().GetErrorString ? rccl().GetErrorString(e) : "";
    throw std::runtime_error(std::string(what) + ": " + (s ? s : "RCCL error"));
  }
}

}  // namespace

struct zkl_comm {
  int device = 0, world = 1, rank = 0;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  void* d_lens = nullptr;  // world x u64
  void* d_buf = nullptr;   // world x cap bytes (this rank's blob in slot `rank`)
  size_t cap = 0;
  double last_ms = 0;      // device time of the last gather (HIP events on the comm stream)
  bool broken = false;     // a failed collective leaves peers mid-call: the comm is not reused
};

namespace {
// RAII for the two timing events and the RCCL group of one gather: an exception between
// ncclGroupStart and ncclGroupEnd still closes the group, and the events never leak.
struct Events {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  Events() {
    ZKL_HIPCHECK(hipEventCreate(&e0));
    ZKL_HIPCHECK(hipEventCreate(&e1));
  }
  ~Events() {
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }
};
struct Group {
  bool open = false;
  void start() {
    nccl_check(rccl().GroupStart(), "ncclGroupStart");
    open = true;
  }
  void end() {
    open = false;
    nccl_check(rccl().GroupEnd(), "ncclGroupEnd");
  }
  ~Group() {
    if (open) (void)rccl().GroupEnd();
  }
};

void ensure_cap(zkl_comm* c, size_t need) {
  if (need <= c->cap) return;
  if (c->d_buf) (void)hipFree(c->d_buf);
  c->d_buf = nullptr;
  c->cap = 0;
  const size_t cap = (need + 4095) & ~(size_t)4095;
  ZKL_HIPCHECK(hipMalloc(&c->d_buf, cap * (size_t)c->world));
  c->cap = cap;
}
}  // namespace

extern "C" {

int zkl_comm_available(void) {
  return zkl::guarded_call([] { (void)rccl(); });
}

int zkl_comm_unique_id(uint8_t id_out[128]) {
  if (!id_out) return ZKL_E_INVALID;
  return zkl::guarded_call([&] {
    ncclUniqueId id;
    nccl_check(rccl().GetUniqueId(&id), "ncclGetUniqueId");
    memcpy(id_out, id.internal, 128);
  });
}

int zkl_comm_init(int device, int world, int rank, const uint8_t id[128], zkl_comm** out) {
  if (!id || !out || world < 1 || rank < 0 || rank >= world) return ZKL_E_INVALID;
  *out = nullptr;
  zkl_comm* c = new zkl_comm;
  c->device = device;
  c->world = world;
  c->rank = rank;
  const int rc = zkl::guarded_call([&] {
    ZKL_HIPCHECK(hipSetDevice(device));
    ZKL_HIPCHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    ZKL_HIPCHECK(hipMalloc(&c->d_lens, sizeof(uint64_t) * (size_t)world));
    ncclUniqueId uid;
    memcpy(uid.internal, id, 128);
    nccl_check(rccl().CommInitRank(&c->comm, world, uid, rank), "ncclCommInitRank");
  });
  if (rc) {
    zkl_comm_destroy(c);
    return rc;
  }
  *out = c;
  return ZKL_OK;
}

int zkl_comm_gather_bytes(zkl_comm* c, const uint8_t* data, size_t len, int root, uint8_t** out, size_t* lens_out) {
  if (!c || (!data && len) || root < 0 || root >= c->world) return ZKL_E_INVALID;
  if (c->rank == root && (!out || !lens_out)) return ZKL_E_INVALID;
  if (c->broken)
    return zkl::guarded_call([] {
      throw std::runtime_error("zkl_comm_gather_bytes: the communicator failed in an earlier collective; destroy it");
    });
  std::vector<uint8_t> host;
  std::vector<uint64_t> lens(c->world, 0);
  const int rc = zkl::guarded_call([&] {
    const Rccl& R = rccl();
    ZKL_HIPCHECK(hipSetDevice(c->device));
    Events ev;
    ZKL_HIPCHECK(hipEventRecord(ev.e0, c->stream));
    // 1. every rank learns every blob length (one u64 per rank)
    const uint64_t mine = len;
    uint8_t* d_lens = (uint8_t*)c->d_lens;
    ZKL_HIPCHECK(hipMemcpyAsync(d_lens + sizeof(uint64_t) * (size_t)c->rank, &mine, sizeof mine,
                                hipMemcpyHostToDevice, c->stream));
    nccl_check(R.AllGather(d_lens + sizeof(uint64_t) * (size_t)c->rank, d_lens, 1, ncclUint64, c->comm, c->stream),
               "ncclAllGather (lengths)");
    ZKL_HIPCHECK(hipMemcpyAsync(lens.data(), d_lens, sizeof(uint64_t) * (size_t)c->world, hipMemcpyDeviceToHost,
                                c->stream));
    ZKL_HIPCHECK(hipStreamSynchronize(c->stream));
    size_t mx = 0;
    for (uint64_t l : lens) mx = std::max<size_t>(mx, (size_t)l);
    ensure_cap(c, std::max<size_t>(mx, 1));
    uint8_t* slot = (uint8_t*)c->d_buf + c->cap * (size_t)c->rank;
    if (len) ZKL_HIPCHECK(hipMemcpyAsync(slot, data, len, hipMemcpyHostToDevice, c->stream));
    // 2. point-to-point to the root, one transfer per rank, grouped so they progress together
    Group group;
    group.start();
    if (c->rank == root) {
      for (int r = 0; r < c->world; r++)
        if (r != root && lens[r])
          nccl_check(R.Recv((uint8_t*)c->d_buf + c->cap * (size_t)r, (size_t)lens[r], ncclUint8, r, c->comm, c->stream),
                     "ncclRecv");
    } else if (len) {
      nccl_check(R.Send(slot, len, ncclUint8, root, c->comm, c->stream), "ncclSend");
    }
    group.end();
    ZKL_HIPCHECK(hipEventRecord(ev.e1, c->stream));
    if (c->rank == root) {
      size_t tot = 0;
      for (uint64_t l : lens) tot += (size_t)l;
      host.resize(tot);
      size_t off = 0;
      for (int r = 0; r < c->world; r++) {
        if (lens[r])
          ZKL_HIPCHECK(hipMemcpyAsync(host.data() + off, (uint8_t*)c->d_buf + c->cap * (size_t)r, (size_t)lens[r],
                                      hipMemcpyDeviceToHost, c->stream));
        off += (size_t)lens[r];
      }
    }
    ZKL_HIPCHECK(hipStreamSynchronize(c->stream));
    float ms = 0;
    ZKL_HIPCHECK(hipEventElapsedTime(&ms, ev.e0, ev.e1));
    c->last_ms = ms;
  });
  if (rc) {
    c->broken = true;
    return rc;
  }
  if (c->rank == root) {
    uint8_t* b = (uint8_t*)malloc(std::max<size_t>(host.size(), 1));
    if (!b) return ZKL_E_OOM;
    if (!host.empty()) memcpy(b, host.data(), host.size());
    *out = b;
    for (int r = 0; r < c->world; r++) lens_out[r] = (size_t)lens[r];
  }
  return ZKL_OK;
}

double zkl_comm_last_ms(const zkl_comm* c) { return c ? c->last_ms : 0.0; }

void zkl_comm_destroy(zkl_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) {
    try {
      (void)rccl().CommDestroy(c->comm);
    } catch (...) {
    }
  }
  if (c->d_buf) (void)hipFree(c->d_buf);
  if (c->d_lens) (void)hipFree(c->d_lens);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

}  // extern "C"
