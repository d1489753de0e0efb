// The reduction "ladder" of the Harris whitepaper shipped with the reference
// (cuda/C/src/reduction/doc/reduction.pdf p.7-35), re-expressed for CDNA wave64.
//
// The reference's CUDA code keeps only "kernel 6" (reduction_kernel.cu:74-253); its --kernel=0..5
// cases are empty stubs that launch nothing (reduction_kernel.cu:276-289, bug B5). The stock
// OpenCL twin still has all seven (oclReduction_kernel.cl:35-273). Here all seven exist, with the
// operator identity for out-of-range lanes (bugs B1/B2 fixed) and a wave64 cross-lane tail
// instead of the 32-lane volatile-LDS lockstep (reduction_kernel.cu:110-122; readme.txt:1-14):
//   0 interleaved addressing, divergent branch     4 + last wave unrolled (shuffles)
//   1 interleaved addressing, strided index        5 + completely unrolled (template BLOCK)
//   2 sequential addressing                        6 + multiple elements per thread (grid-stride,
//   3 + first add during the global load             fixed grid of `max_blocks`) = reference kernel 6
// Multi-pass like benchmarkReduce* (reduction.cpp:344-357): the same kernel is relaunched on the
// partials until one value remains. These exist for parity, teaching and the shmoo; the tuned
// path is the single-pass kernel of reduce.hpp (--kernel=7).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

#include "mireduce/types.hpp"

namespace mireduce {

// First-pass launch geometry, as getNumBlocksAndThreads (reduction.cpp:272-291); any power-of-two
// thread count up to 1024 (blocks narrower than a wave reduce over their active lanes).
void ladder_geometry(int kernel, uint64_t n, int max_threads, int max_blocks, int* blocks, int* threads);

// Bytes of scratch ladder_reduce needs for (kernel, n) — two ping-pong partial buffers.
size_t ladder_scratch_bytes(int kernel, uint64_t n, int max_threads, int max_blocks);

// Enqueue the full multi-pass reduction; result (acc type) in out[0]. `scratch` must hold
// ladder_scratch_bytes(...) bytes. Returns the first-pass grid size.
int ladder_reduce(int kernel, const void* in, uint64_t n, DType t, Op op, DType acc, void* out,
                  void* scratch, int max_threads, int max_blocks, hipStream_t stream);

// The reference's timed multi-pass reduction (benchmarkReduce*, reduction.cpp:319-374): first
// pass, then relaunches on the partials while more than `cpu_thresh` remain (--cputhresh), or none
// at all with `cpu_final` (--cpufinal). `left` == 1: the result is in out[0]; `left` > 1: the
// remaining partials (acc type) are at `partials` (inside scratch) for the caller's host fold.
struct LadderPasses {
  int first_grid = 0;
  int passes = 0;             // kernel launches
  uint64_t left = 0;          // partials remaining
  const void* partials = nullptr;
};
LadderPasses ladder_reduce_passes(int kernel, const void* in, uint64_t n, DType t, Op op, DType acc, void* out,
                                  void* scratch, int max_threads, int max_blocks, uint64_t cpu_thresh,
                                  bool cpu_final, hipStream_t stream);

}  // namespace mireduce
