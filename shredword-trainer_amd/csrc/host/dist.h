// Multi-GPU plumbing: one process per MI355X, RCCL over xGMI.
//
// Two multi-GPU modes (trainer option dist):
//  * replicate (default): the load is sharded -- each rank counts the words of its byte range and
//    the word lists are all-gathered and merged (dist_allgather_bytes, corpus.h) -- and every rank
//    then runs the whole merge loop on the full word table, with no per-merge collective;
//  * exchange: the word table is sharded by contiguous word ranges.  Per merge the
// only exchange is one all-gather of every rank's compacted neighbour-delta records (a fixed
// bucket per rank; a second round only when a bucket overflows), so every rank receives the
// identical record multiset, combines it (sum of weights, min of first touch: order-free) and
// replays the identical heap.  Setup and the rare host-side reductions (initial
// pair lists, final token histogram) go through small device staging buffers.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

#include "selector.h"

namespace shred {

struct DistState {
  int rank = 0;
  int world = 1;
  int device = 0;
  void* comm = nullptr;  // ncclComm_t
};

DistState& dist_state();
inline bool dist_active() { return dist_state().world > 1 && dist_state().comm != nullptr; }

int dist_unique_id(void* out, size_t cap);
int dist_init(int rank, int world, const void* id, size_t len, int device);
// Ranks of the job's communicator (ncclCommCount), 0 without one.
int dist_comm_ranks();
int dist_finalize();

// All-gather of `bytes` per rank (device buffers; recv holds world x bytes) on `stream`, over
// `comm` (an ncclComm_t: the job's, or the single-rank one below).
void dist_allgather_device(void* comm, const void* send, void* recv, size_t bytes, void* stream);
// A single-rank communicator on `device` (tests: runs the multi-GPU exchange path on one GPU).
void* dist_local_comm(int device);
// In-place all-reduce of n u64 device values on `stream` (sum, or min when min_op).
void dist_allreduce_device(uint64_t* dev_buf, size_t n, bool min_op, void* stream);
// Same for host values, staged through a device buffer (synchronous).
void dist_allreduce_host(uint64_t* host, size_t n, bool min_op);
// Every rank's pair list, merged: counts summed, first touch min (synchronous).
void dist_merge_pairs(std::vector<PairCount>* pairs);
// All-gather of a host byte buffer of any size per rank (corpus.h LoadGather): every rank's
// buffer concatenated in rank order, valid until the next call (synchronous).
const void* dist_allgather_bytes(void* ctx, const void* send, size_t nbytes, size_t* out_bytes);

}  // namespace shred
