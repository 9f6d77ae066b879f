// Multi-GPU plumbing over RCCL: see dist.h.
#include "dist.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "common.h"

namespace shred {

namespace {
// RCCL is opened on first use, not linked: a one-GPU process never maps it, and a process that
// already holds one (PyTorch-ROCm's, loaded by torch.distributed) shares that copy.  Two RCCLs
// in one process with torch abort at exit (double free), measured.
struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclCommCount) CommCount = nullptr;
};
const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* n : {"librccl.so", "librccl.so.1"})  // a copy already in the process
      if (!h) h = dlopen(n, RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
    for (const char* n : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
      if (!h) h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
    if (!h) fatal("RCCL (librccl.so.1) could not be loaded: the multi-GPU exchange needs it");
    auto sym = [&](const char* name) {
      void* f = dlsym(h, name);
      if (!f) fatal("RCCL lacks a symbol the exchange uses");
      return f;
    };
    r.GetUniqueId = reinterpret_cast<decltype(r.GetUniqueId)>(sym("ncclGetUniqueId"));
    r.CommInitRank = reinterpret_cast<decltype(r.CommInitRank)>(sym("ncclCommInitRank"));
    r.CommInitAll = reinterpret_cast<decltype(r.CommInitAll)>(sym("ncclCommInitAll"));
    r.CommDestroy = reinterpret_cast<decltype(r.CommDestroy)>(sym("ncclCommDestroy"));
    r.AllGather = reinterpret_cast<decltype(r.AllGather)>(sym("ncclAllGather"));
    r.AllReduce = reinterpret_cast<decltype(r.AllReduce)>(sym("ncclAllReduce"));
    r.GetErrorString = reinterpret_cast<decltype(r.GetErrorString)>(sym("ncclGetErrorString"));
    r.CommCount = reinterpret_cast<decltype(r.CommCount)>(sym("ncclCommCount"));
  });
  return r;
}

void nccl_ok(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    std::fprintf(stderr, "[ERROR]\t RCCL %s failed: %s\n", what, rccl().GetErrorString(r));
    std::fflush(stderr);
    std::abort();
  }
}
void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    std::fprintf(stderr, "[ERROR]\t HIP %s failed: %s\n", what, hipGetErrorString(e));
    std::fflush(stderr);
    std::abort();
  }
}
}  // namespace

DistState& dist_state() {
  static DistState s;
  return s;
}

int dist_unique_id(void* out, size_t cap) {
  if (cap < sizeof(ncclUniqueId)) return -1;
  ncclUniqueId id;
  if (rccl().GetUniqueId(&id) != ncclSuccess) return -1;
  std::memcpy(out, &id, sizeof(id));
  return (int)sizeof(id);
}

int dist_init(int rank, int world, const void* id, size_t len, int device) {
  DistState& s = dist_state();
  if (world <= 1) {
    s = DistState();
    s.device = device;
    return 0;
  }
  if (len < sizeof(ncclUniqueId) || rank < 0 || rank >= world) return -1;
  hip_ok(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm;
  if (rccl().CommInitRank(&comm, world, uid, rank) != ncclSuccess) return -1;
  s.rank = rank;
  s.world = world;
  s.device = device;
  s.comm = comm;
  return 0;
}

int dist_comm_ranks() {
  const DistState& s = dist_state();
  if (!s.comm) return 0;
  int n = 0;
  nccl_ok(rccl().CommCount((ncclComm_t)s.comm, &n), "ncclCommCount");
  return n;
}

int dist_finalize() {
  DistState& s = dist_state();
  if (s.comm) rccl().CommDestroy((ncclComm_t)s.comm);
  s = DistState();
  return 0;
}

void dist_allgather_device(void* comm, const void* send, void* recv, size_t bytes, void* stream) {
  nccl_ok(rccl().AllGather(send, recv, bytes, ncclUint8, (ncclComm_t)comm, (hipStream_t)stream), "ncclAllGather");
}

void* dist_local_comm(int device) {
  static std::unordered_map<int, ncclComm_t> comms;
  auto it = comms.find(device);
  if (it != comms.end()) return it->second;
  hip_ok(hipSetDevice(device), "hipSetDevice");
  ncclComm_t comm;
  int dev = device;
  nccl_ok(rccl().CommInitAll(&comm, 1, &dev), "ncclCommInitAll");
  comms.emplace(device, comm);
  return comm;
}

void dist_allreduce_device(uint64_t* buf, size_t n, bool min_op, void* stream) {
  if (!dist_active() || n == 0) return;
  nccl_ok(rccl().AllReduce(buf, buf, n, ncclUint64, min_op ? ncclMin : ncclSum, (ncclComm_t)dist_state().comm,
                        (hipStream_t)stream),
          "ncclAllReduce");
}

void dist_allreduce_host(uint64_t* host, size_t n, bool min_op) {
  if (!dist_active() || n == 0) return;
  hip_ok(hipSetDevice(dist_state().device), "hipSetDevice");
  void* d = nullptr;
  hip_ok(hipMalloc(&d, n * sizeof(uint64_t)), "hipMalloc");
  hip_ok(hipMemcpy(d, host, n * sizeof(uint64_t), hipMemcpyHostToDevice), "hipMemcpy");
  dist_allreduce_device((uint64_t*)d, n, min_op, nullptr);
  hip_ok(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
  hip_ok(hipMemcpy(host, d, n * sizeof(uint64_t), hipMemcpyDeviceToHost), "hipMemcpy");
  hip_ok(hipFree(d), "hipFree");
}

void dist_merge_pairs(std::vector<PairCount>* pairs) {
  if (!dist_active()) return;
  DistState& s = dist_state();
  uint64_t n = pairs->size();
  uint64_t maxn = n;
  {
    uint64_t v = maxn;
    // max via min of the negation
    uint64_t neg = ~v;
    dist_allreduce_host(&neg, 1, true);
    maxn = ~neg;
  }
  const size_t rec = sizeof(PairCount);
  const size_t bytes = (size_t)(maxn + 1) * rec;  // first record carries the count
  std::vector<uint8_t> send(bytes, 0);
  PairCount head{};
  head.count = n;
  std::memcpy(send.data(), &head, rec);
  if (n) std::memcpy(send.data() + rec, pairs->data(), n * rec);
  hip_ok(hipSetDevice(s.device), "hipSetDevice");
  void *dsend = nullptr, *drecv = nullptr;
  hip_ok(hipMalloc(&dsend, bytes), "hipMalloc");
  hip_ok(hipMalloc(&drecv, bytes * s.world), "hipMalloc");
  hip_ok(hipMemcpy(dsend, send.data(), bytes, hipMemcpyHostToDevice), "hipMemcpy");
  nccl_ok(rccl().AllGather(dsend, drecv, bytes, ncclUint8, (ncclComm_t)s.comm, nullptr), "ncclAllGather");
  hip_ok(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
  std::vector<uint8_t> recv(bytes * s.world);
  hip_ok(hipMemcpy(recv.data(), drecv, recv.size(), hipMemcpyDeviceToHost), "hipMemcpy");
  hip_ok(hipFree(dsend), "hipFree");
  hip_ok(hipFree(drecv), "hipFree");
  std::unordered_map<uint64_t, size_t> at;
  std::vector<PairCount> out;
  for (int r = 0; r < s.world; ++r) {
    const uint8_t* blk = recv.data() + (size_t)r * bytes;
    PairCount h;
    std::memcpy(&h, blk, rec);
    for (uint64_t i = 0; i < h.count; ++i) {
      PairCount p;
      std::memcpy(&p, blk + (i + 1) * rec, rec);
      const uint64_t k = pack_pair(p.a, p.b);
      auto it = at.find(k);
      if (it == at.end()) {
        at.emplace(k, out.size());
        out.push_back(p);
      } else {
        out[it->second].count += p.count;
        out[it->second].ft = std::min(out[it->second].ft, p.ft);
      }
    }
  }
  pairs->swap(out);
}

}  // namespace shred

namespace shred {

const void* dist_allgather_bytes(void*, const void* send, size_t nbytes, size_t* out_bytes) {
  static std::vector<uint8_t> keep;
  DistState& s = dist_state();
  keep.clear();
  if (!dist_active()) {
    keep.assign((const uint8_t*)send, (const uint8_t*)send + nbytes);
    keep.push_back(0);  // never NULL: NULL means a failed gather
    *out_bytes = nbytes;
    return keep.data();
  }
  uint64_t neg = ~(uint64_t)nbytes;  // max via min of the negation
  dist_allreduce_host(&neg, 1, true);
  const size_t top = (size_t)~neg;
  const size_t slot = 8 + top;  // [u64 size][payload, padded to the largest]
  std::vector<uint8_t> mine(slot, 0);
  const uint64_t n64 = nbytes;
  std::memcpy(mine.data(), &n64, 8);
  if (nbytes) std::memcpy(mine.data() + 8, send, nbytes);
  hip_ok(hipSetDevice(s.device), "hipSetDevice");
  void *dsend = nullptr, *drecv = nullptr;
  hip_ok(hipMalloc(&dsend, slot), "hipMalloc");
  hip_ok(hipMalloc(&drecv, slot * s.world), "hipMalloc");
  hip_ok(hipMemcpy(dsend, mine.data(), slot, hipMemcpyHostToDevice), "hipMemcpy");
  nccl_ok(rccl().AllGather(dsend, drecv, slot, ncclUint8, (ncclComm_t)s.comm, nullptr), "ncclAllGather");
  hip_ok(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
  std::vector<uint8_t> all(slot * s.world);
  hip_ok(hipMemcpy(all.data(), drecv, all.size(), hipMemcpyDeviceToHost), "hipMemcpy");
  hip_ok(hipFree(dsend), "hipFree");
  hip_ok(hipFree(drecv), "hipFree");
  for (int r = 0; r < s.world; ++r) {
    uint64_t n = 0;
    std::memcpy(&n, all.data() + (size_t)r * slot, 8);
    keep.insert(keep.end(), all.data() + (size_t)r * slot + 8, all.data() + (size_t)r * slot + 8 + n);
  }
  *out_bytes = keep.size();
  static const uint8_t kNothing = 0;  // NULL means a failed gather (shred_gather_fn)
  return keep.empty() ? &kNothing : keep.data();
}

}  // namespace shred
