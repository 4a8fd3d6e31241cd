// TEST INFRASTRUCTURE ONLY -- an NCCL-ABI library over POSIX shared memory, so that the
// multi-rank branches of zkl_comm_gather_bytes (csrc/comm.cpp: the root's ncclRecv loop, the
// non-root ncclSend, zero and unequal lengths, capacity growth, the `broken` path) run with
// several processes on ONE GPU, where real RCCL refuses duplicate devices.  Selected with
// ZKL_RCCL_LIB=<this .so> (comm.cpp dlopens it instead of librccl.so.1); tests/test_comm_stub.py.
//
// Semantics: every call runs eagerly on the host.  The caller's stream is synchronised, device
// buffers are copied through host memory, and ranks meet in a shared-memory segment named by the
// unique id: an all-gather area (round counters per rank) and one mailbox per (src, dst) pair
// (a send waits for the mailbox to be empty, a receive for it to be full).  Group calls are no-ops.
// A wait longer than ZKL_NCCL_STUB_TIMEOUT_S (default 30) fails the call.  Fault injection:
// ZKL_NCCL_STUB_FAIL=<allgather|send|recv> with ZKL_NCCL_STUB_FAIL_RANK=<r> makes that call on rank
// r return an error.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

namespace {
constexpr int MAXW = 8;
constexpr size_t AG_BYTES = 256;         // per-rank all-gather contribution
constexpr size_t BOX_BYTES = 64u << 20;  // one mailbox
typedef int ncclResult_t;
enum { ncclSuccess = 0, ncclUnhandledCudaError = 1, ncclSystemError = 2, ncclInvalidArgument = 4 };

struct Box {
  std::atomic<uint64_t> sent, taken;
  uint64_t len;
};
struct Shm {
  std::atomic<uint32_t> joined;
  std::atomic<uint64_t> ag_in[MAXW], ag_out[MAXW];  // all-gather rounds written / read, per rank
  uint8_t ag[MAXW][AG_BYTES];
  Box box[MAXW][MAXW];  // [src][dst]
};
size_t shm_bytes(int world) { return sizeof(Shm) + (size_t)world * world * BOX_BYTES; }

thread_local std::string g_err;

double timeout_s() {
  const char* e = getenv("ZKL_NCCL_STUB_TIMEOUT_S");
  return e ? atof(e) : 30.0;
}
template <class F>
bool wait_until(F&& ready) {
  const auto t0 = std::chrono::steady_clock::now();
  const double lim = timeout_s();
  while (!ready()) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  return true;
}
bool inject(const char* op, int rank) {
  const char* f = getenv("ZKL_NCCL_STUB_FAIL");
  const char* r = getenv("ZKL_NCCL_STUB_FAIL_RANK");
  return f && !strcmp(f, op) && (!r || atoi(r) == rank);
}
size_t type_size(int t) { return t == 5 || t == 4 || t == 7 ? 8 : t == 2 || t == 3 || t == 6 ? 4 : 1; }
ncclResult_t fail(ncclResult_t e, const std::string& m) {
  g_err = m;
  fprintf(stderr, "[nccl stub] %s\n", m.c_str());
  return e;
}
}  // namespace

struct ncclComm {
  Shm* shm = nullptr;
  int world = 1, rank = 0;
  uint64_t ag_round = 0;
  std::string name;
};
typedef struct ncclComm* ncclComm_t;
typedef struct { char internal[128]; } ncclUniqueId;

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
  static thread_local std::string s;
  s = "nccl stub error " + std::to_string(r) + (g_err.empty() ? "" : ": " + g_err);
  return s.c_str();
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  memset(id->internal, 0, sizeof id->internal);
  uint64_t r[2] = {(uint64_t)getpid(), (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count()};
  FILE* f = fopen("/dev/urandom", "rb");
  if (f) {
    if (fread(r, 1, sizeof r, f) != sizeof r) r[1] ^= 0x9E3779B97F4A7C15ull;
    fclose(f);
  }
  snprintf(id->internal, sizeof id->internal, "/zkl_nccl_stub_%016llx%016llx", (unsigned long long)r[0],
           (unsigned long long)r[1]);
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int world, ncclUniqueId id, int rank) {
  if (world < 1 || world > MAXW || rank < 0 || rank >= world) return fail(ncclInvalidArgument, "bad world/rank");
  ncclComm* c = new ncclComm;
  c->world = world;
  c->rank = rank;
  c->name.assign(id.internal, strnlen(id.internal, sizeof id.internal));
  int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0) { delete c; return fail(ncclSystemError, "shm_open " + c->name); }
  const size_t bytes = shm_bytes(world);
  if (ftruncate(fd, (off_t)bytes) != 0) { close(fd); delete c; return fail(ncclSystemError, "ftruncate"); }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) { delete c; return fail(ncclSystemError, "mmap"); }
  c->shm = (Shm*)p;
  c->shm->joined.fetch_add(1);
  if (!wait_until([&] { return c->shm->joined.load() >= (uint32_t)world; })) {
    munmap(p, bytes);
    delete c;
    return fail(ncclSystemError, "timed out waiting for the other ranks to join");
  }
  *out = c;
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclSuccess;
  if (c->shm) munmap(c->shm, shm_bytes(c->world));
  shm_unlink(c->name.c_str());  // every rank mapped it before init returned; later unlinks fail harmlessly
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, int type, ncclComm_t c, hipStream_t s) {
  if (inject("allgather", c->rank)) return fail(ncclSystemError, "injected allgather failure");
  const size_t b = count * type_size(type);
  if (b > AG_BYTES) return fail(ncclInvalidArgument, "all-gather contribution too large for the stub");
  if (hipStreamSynchronize(s) != hipSuccess) return fail(ncclUnhandledCudaError, "hipStreamSynchronize");
  Shm* m = c->shm;
  const uint64_t r = ++c->ag_round;
  // the previous round's area may be reused once every rank has read it
  if (!wait_until([&] {
        for (int k = 0; k < c->world; k++)
          if (m->ag_out[k].load() < r - 1) return false;
        return true;
      }))
    return fail(ncclSystemError, "all-gather: timed out waiting for the previous round");
  if (hipMemcpy(m->ag[c->rank], send, b, hipMemcpyDeviceToHost) != hipSuccess)
    return fail(ncclUnhandledCudaError, "hipMemcpy D2H");
  m->ag_in[c->rank].store(r);
  if (!wait_until([&] {
        for (int k = 0; k < c->world; k++)
          if (m->ag_in[k].load() < r) return false;
        return true;
      }))
    return fail(ncclSystemError, "all-gather: timed out waiting for the other ranks");
  std::vector<uint8_t> all(b * c->world);
  for (int k = 0; k < c->world; k++) memcpy(all.data() + b * k, m->ag[k], b);
  m->ag_out[c->rank].store(r);
  if (hipMemcpy(recv, all.data(), all.size(), hipMemcpyHostToDevice) != hipSuccess)
    return fail(ncclUnhandledCudaError, "hipMemcpy H2D");
  return ncclSuccess;
}

ncclResult_t ncclSend(const void* buf, size_t count, int type, int peer, ncclComm_t c, hipStream_t s) {
  if (inject("send", c->rank)) return fail(ncclSystemError, "injected send failure");
  const size_t b = count * type_size(type);
  if (peer < 0 || peer >= c->world || b > BOX_BYTES) return fail(ncclInvalidArgument, "send: bad peer or size");
  if (hipStreamSynchronize(s) != hipSuccess) return fail(ncclUnhandledCudaError, "hipStreamSynchronize");
  Box& x = c->shm->box[c->rank][peer];
  if (!wait_until([&] { return x.taken.load() == x.sent.load(); })) return fail(ncclSystemError, "send: mailbox full");
  uint8_t* data = (uint8_t*)(c->shm + 1) + ((size_t)c->rank * c->world + peer) * BOX_BYTES;
  if (hipMemcpy(data, buf, b, hipMemcpyDeviceToHost) != hipSuccess) return fail(ncclUnhandledCudaError, "hipMemcpy D2H");
  x.len = b;
  x.sent.fetch_add(1);
  return ncclSuccess;
}

ncclResult_t ncclRecv(void* buf, size_t count, int type, int peer, ncclComm_t c, hipStream_t s) {
  if (inject("recv", c->rank)) return fail(ncclSystemError, "injected recv failure");
  const size_t b = count * type_size(type);
  if (peer < 0 || peer >= c->world) return fail(ncclInvalidArgument, "recv: bad peer");
  if (hipStreamSynchronize(s) != hipSuccess) return fail(ncclUnhandledCudaError, "hipStreamSynchronize");
  Box& x = c->shm->box[peer][c->rank];
  if (!wait_until([&] { return x.sent.load() > x.taken.load(); }))
    return fail(ncclSystemError, "recv: timed out waiting for rank " + std::to_string(peer));
  if (x.len != b) return fail(ncclInvalidArgument, "recv: size differs from the matching send");
  const uint8_t* data = (const uint8_t*)(c->shm + 1) + ((size_t)peer * c->world + c->rank) * BOX_BYTES;
  if (hipMemcpy(buf, data, b, hipMemcpyHostToDevice) != hipSuccess) return fail(ncclUnhandledCudaError, "hipMemcpy H2D");
  x.taken.fetch_add(1);
  return ncclSuccess;
}

}  // extern "C"
