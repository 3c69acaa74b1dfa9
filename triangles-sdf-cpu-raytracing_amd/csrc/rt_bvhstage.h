// rt_bvhstage.h -- host side of the device BVH build's stage loop
// (rt_bvhgpu.hip): createNode's candidate FIFO (triangles_raytracing.cpp:
// 155-225) for every open node of a stage, and the per-stage work tables the
// device kernels read. Compiled by g++ with OpenMP (rt_bvhstage.cpp): the open
// nodes of a stage are independent, so both the table build and the FIFO run
// over them in parallel, with prefix sums putting every output where the
// serial loop would (same node ids, same child order, same next-stage order).
#pragma once
#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

#include "rt_host.h"

namespace rth {
namespace bvhs {

struct Task {
  uint32_t s, e;  // triangle range [s, e) of one candidate (or one child range)
};
struct Seg {
  uint32_t first, last;  // position range in the 3n-element space (axis a: [a*n, (a+1)*n))
  int32_t depth;         // remaining introsort depth
  uint32_t pad;
};
struct SahChunk {
  uint32_t task, axis, lo, hi;  // triangle range [lo, hi) of candidate `task` on `axis`
  uint32_t group;               // task * 3 + axis
};
struct SahGroup {
  uint32_t first, count;  // its chunks
};
struct Cand {
  uint32_t lo, hi;  // index units
};
// createNode's state of one node: its range, ChipQueue contents (FIFO) and
// dividers. A node splits at most 7 times and its queue is dropped at the 7th
// split, so the queue never holds more than 8 candidates (a layer of 4 that
// all split reaches 7 splits).
struct OpenState {
  uint32_t start, end;  // index units
  uint32_t qn;
  int32_t nd;
  Cand q[8];
  uint32_t div[8];
};

// An anonymous mapping of a capacity bound with transparent huge pages
// requested: the build writes each element once, and fresh 4 KiB pages of
// std::vector growth cost more than the stage logic itself (untouched pages
// of the reservation cost nothing). Elements are not constructed.
template <class T>
struct Arena {
  T *p = nullptr;
  size_t cap = 0, bytes = 0;
  Arena() = default;
  Arena(const Arena &) = delete;
  Arena &operator=(const Arena &) = delete;
  ~Arena();
  bool reserve(size_t c);
  T &operator[](size_t i) { return p[i]; }
  const T &operator[](size_t i) const { return p[i]; }
};

struct Stage {
  uint32_t n = 0;      // triangles
  uint32_t chunk = 0;  // SAH chunk length (triangles)
  // nodes (createNode's m_nodes) and per-node FIFO state, indexed by node id
  Arena<BvhHostNode> H;
  Arena<OpenState> OS;
  size_t n_nodes = 0;
  // open nodes of this stage / the next one
  Arena<int32_t> open, next;
  size_t n_open = 0, n_next = 0;
  // child ranges (triangle units) of completed nodes, and (node, child slot) per range
  Arena<Task> ranges;
  Arena<std::pair<int32_t, int32_t>> range_of;
  size_t n_ranges = 0;

  // this stage's work: every queued candidate of every open node that
  // tryDivide sorts (> 8 triangles) is a task
  std::vector<Task> tasks;
  std::vector<int32_t> task_of;    // task of open node o's candidate c: task_of[task_off[o] + c] (-1: not sorted)
  std::vector<uint32_t> task_off;  // per open node
  std::vector<SahChunk> ch;        // [axis-0 chunks of all tasks | axis 1 | axis 2]
  std::vector<SahGroup> grp;       // per (task, axis): 3 task + axis
  std::vector<Seg> segs;           // the sorts: [axis 0 of all tasks | axis 1 | axis 2]
  std::vector<float> cost;         // per (task, axis): best SAH cost
  std::vector<uint32_t> dvd;       // and its divider (triangle units)
  std::vector<uint32_t> action;    // per task: 0 keep X order, 1 Y, 2 Z, 3 restore
  uint32_t nc_axis = 0;            // chunks per axis

  bool init(uint32_t ntri, uint32_t chunk_len);
  void prologue();
  // first minimum over each (task, axis)'s chunks of (cost, divider)
  void reduce_sah(const float *ccost, const uint32_t *cdiv);
  // createNode's FIFO for every open node (after the stage's SAH results);
  // false when a bound is exceeded (err says which)
  bool fifo(std::string &err);
  void advance() {
    std::swap(open.p, next.p);
    std::swap(open.cap, next.cap);
    std::swap(open.bytes, next.bytes);
    n_open = n_next;
    n_next = 0;
  }

 private:
  std::vector<uint32_t> a_, b_, kind_;  // per open node scratch
};

// The device builder's stage loop with its device steps done on the host
// (stage copies, std::sort of every segment, the chunked SAH sweeps, the
// apply, child boxes): checks the host half (prologue / reduce_sah / fifo, in
// parallel) against the host builder on machines without a GPU, and under
// the sanitizers. Same tree as build_bvh8.
bool emulate_device_build(const float *vpos4, int64_t nverts, const uint32_t *idx, int64_t nidx, BVHGpu &out,
                          std::string &err, unsigned want = kBvhAll);
}  // namespace bvhs
}  // namespace rth
