// Multi-GPU exchange of the sharded scans on RCCL over xGMI, behind the C ABI:
// one process per GPU, a communicator per process.  The scan shards with no collective on its hot
// path; the exchanges are the one-off all-gather of the packed genotype shards, the broadcast of
// P / Py from rank 0, and the gather of the hit records at the end (replaces the reference's
// separate parallel=[N,k] processes that each write out_file.k: remma_epiAA.py:109-161).
//
// Host buffers in, host buffers out: each call stages through device memory on the
// communicator's stream and returns when the result is on the host.  The unique id that seeds the
// communicator is created by rank 0 (gmat_comm_unique_id) and shared by the launcher (a file for
// single-node runs, gmat_amd/dist.py).
#include <rccl/rccl.h>

#include <algorithm>

#include "common.h"

using namespace gmat;

struct gmat_comm {
  ncclComm_t nc = nullptr;
  int rank = 0, size = 1;
  hipStream_t s = nullptr;
  DBuf a, b;  // staging
  ~gmat_comm() {
    if (nc) (void)ncclCommDestroy(nc);
    if (s) (void)hipStreamDestroy(s);
  }
};

#define GMAT_NCCL(x)                                                                            \
  do {                                                                                          \
    ncclResult_t r_ = (x);                                                                      \
    if (r_ != ncclSuccess) {                                                                    \
      ::gmat::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #x, ncclGetErrorString(r_));     \
      return GMAT_E_HIP;                                                                        \
    }                                                                                           \
  } while (0)

extern "C" int gmat_comm_unique_id(uint8_t *out128) {
  GMAT_CHECK(out128, GMAT_E_ARG, "gmat_comm_unique_id: null");
  ncclUniqueId id;
  GMAT_NCCL(ncclGetUniqueId(&id));
  memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
  return GMAT_OK;
}

extern "C" int gmat_comm_init(gmat_comm **out, int nranks, int rank, const uint8_t *id128) {
  GMAT_CHECK(out && id128 && nranks >= 1 && rank >= 0 && rank < nranks, GMAT_E_ARG, "gmat_comm_init: bad arguments");
  auto *c = new gmat_comm();
  c->rank = rank;
  c->size = nranks;
  ncclUniqueId id;
  memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
  if (hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    set_error("gmat_comm_init: stream");
    return GMAT_E_HIP;
  }
  const ncclResult_t r = ncclCommInitRank(&c->nc, nranks, id, rank);
  if (r != ncclSuccess) {
    c->nc = nullptr;
    delete c;
    set_error("ncclCommInitRank: %s", ncclGetErrorString(r));
    return GMAT_E_HIP;
  }
  *out = c;
  return GMAT_OK;
}

extern "C" int gmat_comm_destroy(gmat_comm *c) {
  delete c;
  return GMAT_OK;
}

// recv (size x bytes, rank order) = every rank's send (bytes)
extern "C" int gmat_comm_allgather(gmat_comm *c, const void *send, void *recv, int64_t bytes) {
  GMAT_CHECK(c && send && recv && bytes >= 0, GMAT_E_ARG, "gmat_comm_allgather: bad arguments");
  if (bytes == 0) return GMAT_OK;
  GMAT_TRY(c->a.alloc((size_t)bytes));
  GMAT_TRY(c->b.alloc((size_t)bytes * c->size));
  GMAT_HIP(hipMemcpyAsync(c->a.p, send, bytes, hipMemcpyHostToDevice, c->s));
  GMAT_NCCL(ncclAllGather(c->a.p, c->b.p, (size_t)bytes, ncclUint8, c->nc, c->s));
  GMAT_HIP(hipMemcpyAsync(recv, c->b.p, (size_t)bytes * c->size, hipMemcpyDeviceToHost, c->s));
  GMAT_HIP(hipStreamSynchronize(c->s));
  return GMAT_OK;
}

// buf (bytes) from root to every rank, in place
extern "C" int gmat_comm_broadcast(gmat_comm *c, void *buf, int64_t bytes, int root) {
  GMAT_CHECK(c && buf && bytes >= 0 && root >= 0 && root < c->size, GMAT_E_ARG, "gmat_comm_broadcast: bad arguments");
  if (bytes == 0) return GMAT_OK;
  GMAT_TRY(c->a.alloc((size_t)bytes));
  if (c->rank == root) GMAT_HIP(hipMemcpyAsync(c->a.p, buf, bytes, hipMemcpyHostToDevice, c->s));
  GMAT_NCCL(ncclBroadcast(c->a.p, c->a.p, (size_t)bytes, ncclUint8, root, c->nc, c->s));
  GMAT_HIP(hipMemcpyAsync(buf, c->a.p, bytes, hipMemcpyDeviceToHost, c->s));
  GMAT_HIP(hipStreamSynchronize(c->s));
  return GMAT_OK;
}

// v[k] = op over ranks (op 0 = sum, 1 = max) of v[k], fp64, in place
extern "C" int gmat_comm_allreduce_f64(gmat_comm *c, double *v, int64_t count, int op) {
  GMAT_CHECK(c && v && count >= 0 && (op == 0 || op == 1), GMAT_E_ARG, "gmat_comm_allreduce_f64: bad arguments");
  if (count == 0) return GMAT_OK;
  GMAT_TRY(c->a.alloc((size_t)count * 8));
  GMAT_HIP(hipMemcpyAsync(c->a.p, v, count * 8, hipMemcpyHostToDevice, c->s));
  GMAT_NCCL(ncclAllReduce(c->a.p, c->a.p, (size_t)count, ncclFloat64, op ? ncclMax : ncclSum, c->nc, c->s));
  GMAT_HIP(hipMemcpyAsync(v, c->a.p, count * 8, hipMemcpyDeviceToHost, c->s));
  GMAT_HIP(hipStreamSynchronize(c->s));
  return GMAT_OK;
}

// Gather variable-length byte records to root: counts (size entries) is filled on every rank;
// root's recv receives the ranks' payloads back to back in rank order (recv_cap bytes available).
// The capacity check is collective: root's verdict travels with the counts' all-reduce, so when
// recv is too small EVERY rank returns GMAT_E_OVERFLOW (with *needed set) before any point-to-point
// call is posted.  Point-to-point sends inside one group; the group is always closed, also on error.
extern "C" int gmat_comm_gatherv(gmat_comm *c, const void *send, int64_t bytes, int root, int64_t *counts, void *recv,
                                 int64_t recv_cap, int64_t *needed) {
  GMAT_CHECK(c && counts && bytes >= 0 && (bytes == 0 || send) && root >= 0 && root < c->size, GMAT_E_ARG,
             "gmat_comm_gatherv: bad arguments");
  // [0, size): byte counts; [size]: root's capacity (other ranks add 0)
  std::vector<double> cnt(c->size + 1, 0.0);
  cnt[c->rank] = (double)bytes;
  if (c->rank == root) cnt[c->size] = recv ? (double)recv_cap : 0.0;
  GMAT_TRY(gmat_comm_allreduce_f64(c, cnt.data(), c->size + 1, 0));
  int64_t total = 0;
  for (int r = 0; r < c->size; ++r) {
    counts[r] = (int64_t)cnt[r];
    total += counts[r];
  }
  if (needed) *needed = total;
  GMAT_CHECK((int64_t)cnt[c->size] >= total, GMAT_E_OVERFLOW, "gmat_comm_gatherv: %lld bytes needed, root has %lld",
             (long long)total, (long long)cnt[c->size]);
  if (total == 0) return GMAT_OK;
  GMAT_TRY(c->a.alloc((size_t)std::max<int64_t>(bytes, 1)));
  if (bytes) GMAT_HIP(hipMemcpyAsync(c->a.p, send, bytes, hipMemcpyHostToDevice, c->s));
  if (c->rank == root) GMAT_TRY(c->b.alloc((size_t)total));
  // enqueue inside the group; the first failure is kept and the group closed before returning
  std::string err;
  GMAT_NCCL(ncclGroupStart());
  if (c->rank == root) {
    int64_t off = 0;
    for (int r = 0; r < c->size && err.empty(); ++r) {
      if (counts[r] > 0) {
        if (r == root) {
          const hipError_t he =
              hipMemcpyAsync(c->b.as<uint8_t>() + off, c->a.p, counts[r], hipMemcpyDeviceToDevice, c->s);
          if (he != hipSuccess) err = std::string("hipMemcpyAsync: ") + hipGetErrorString(he);
        } else {
          const ncclResult_t nr = ncclRecv(c->b.as<uint8_t>() + off, (size_t)counts[r], ncclUint8, r, c->nc, c->s);
          if (nr != ncclSuccess) err = std::string("ncclRecv: ") + ncclGetErrorString(nr);
        }
      }
      off += counts[r];
    }
  } else if (bytes > 0) {
    const ncclResult_t nr = ncclSend(c->a.p, (size_t)bytes, ncclUint8, root, c->nc, c->s);
    if (nr != ncclSuccess) err = std::string("ncclSend: ") + ncclGetErrorString(nr);
  }
  const ncclResult_t ge = ncclGroupEnd();
  GMAT_CHECK(err.empty(), GMAT_E_HIP, "gmat_comm_gatherv: %s", err.c_str());
  GMAT_CHECK(ge == ncclSuccess, GMAT_E_HIP, "gmat_comm_gatherv: ncclGroupEnd -> %s", ncclGetErrorString(ge));
  if (c->rank == root) GMAT_HIP(hipMemcpyAsync(recv, c->b.p, total, hipMemcpyDeviceToHost, c->s));
  GMAT_HIP(hipStreamSynchronize(c->s));
  return GMAT_OK;
}

extern "C" int gmat_comm_barrier(gmat_comm *c) {
  double one = 1.0;
  return gmat_comm_allreduce_f64(c, &one, 1, 0);
}
