/*!
 * \file device_reducer.h
 * \brief User-defined reductions that run on the GPU (compile the including file with hipcc).
 *
 * The reference's `rabit::Reducer<DType, freduce>` (`include/rabit/rabit.h:352-394`) runs a host
 * function over struct elements.  For HBM buffers that would mean staging every byte through
 * host memory, so the device form instantiates the reduction as a gfx950 kernel in the user's
 * translation unit and hands the engine a launcher; the engine moves bytes exactly as for the
 * built-in ops (direct IPC transport or RCCL all-to-all + all-gather) and calls the kernel for
 * the reduction step.  The same functor is compiled for the host, so host buffers work too.
 *
 *   struct ArgMax { float v; int idx; };
 *   struct ArgMaxOp {
 *     __host__ __device__ void operator()(ArgMax &dst, const ArgMax &src) const {
 *       if (src.v > dst.v || (src.v == dst.v && src.idx < dst.idx)) dst = src;
 *     }
 *   };
 *   rabit::DeviceReducer<ArgMax, ArgMaxOp> red;
 *   red.Allreduce(d_buf, n);   // d_buf in HBM (or host memory)
 *
 * The reduction must be commutative and associative (as for every rabit reducer).
 */
#ifndef RABIT_DEVICE_REDUCER_H_
#define RABIT_DEVICE_REDUCER_H_

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "rabit/rabit.h"

namespace rabit {
namespace device_reducer_detail {

constexpr int kMaxSources = 8;

struct Sources {
  const void *p[kMaxSources];
};

template <typename DType, typename Op>
__global__ __launch_bounds__(256) void ReduceKernel(DType *dst, Sources srcs, int nsrc, size_t n,
                                                    const int *guard) {
  if (guard != nullptr &&
      __hip_atomic_load(guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
    return;
  }
  const Op op{};
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    DType acc = static_cast<const DType *>(srcs.p[0])[i];
    for (int k = 1; k < nsrc; ++k) op(acc, static_cast<const DType *>(srcs.p[k])[i]);
    dst[i] = acc;
  }
}

/*! \brief engine::IEngine::DeviceReduceLauncher for (DType, Op) */
template <typename DType, typename Op>
int Launch(void *dst, const void *const *srcs, int nsrc, size_t count, const int *guard,
           void *stream) {
  if (nsrc < 1 || nsrc > kMaxSources) return static_cast<int>(hipErrorInvalidValue);
  if (count == 0) return static_cast<int>(hipSuccess);
  Sources s;
  for (int k = 0; k < kMaxSources; ++k) s.p[k] = k < nsrc ? srcs[k] : nullptr;
  // 8 workgroups per CU on 256 CUs, grid-stride beyond that
  size_t blocks = (count + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL((ReduceKernel<DType, Op>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), static_cast<DType *>(dst), s, nsrc, count,
                     guard);
  return static_cast<int>(hipGetLastError());
}

/*! \brief MPI-style host reduce function for host buffers */
template <typename DType, typename Op>
void HostReduce(const void *src, void *dst, int len, const MPI::Datatype &) {
  const Op op{};
  const DType *s = static_cast<const DType *>(src);
  DType *d = static_cast<DType *>(dst);
  for (int i = 0; i < len; ++i) op(d[i], s[i]);
}

template <typename F>
void InvokeLambda(void *fun) {
  (*static_cast<F *>(fun))();
}
}  // namespace device_reducer_detail

/*!
 * \brief reducer of DType elements with a __host__ __device__ functor Op (see file comment).
 *        Works on HBM and host buffers, with the same fault-tolerance semantics as every
 *        rabit collective (the prepare function is skipped when the result is recovered).
 */
template <typename DType, typename Op>
class DeviceReducer {
 public:
  void Allreduce(DType *sendrecvbuf, size_t count, void (*prepare_fun)(void *) = nullptr,
                 void *prepare_arg = nullptr, const char *_file = _FILE, const int _line = _LINE,
                 const char *_caller = _CALLER) {
    engine::GetEngine()->AllreduceDevice(
        sendrecvbuf, sizeof(DType), count, &device_reducer_detail::Launch<DType, Op>,
        &device_reducer_detail::HostReduce<DType, Op>, prepare_fun, prepare_arg, _file, _line,
        _caller);
  }
  /*! \brief lazy-prepare form: prepare() runs right before the reduction unless recovered */
  template <typename F>
  void Allreduce(DType *sendrecvbuf, size_t count, F prepare, const char *_file = _FILE,
                 const int _line = _LINE, const char *_caller = _CALLER) {
    Allreduce(sendrecvbuf, count, &device_reducer_detail::InvokeLambda<F>, &prepare, _file, _line,
              _caller);
  }
};
}  // namespace rabit
#endif  // RABIT_DEVICE_REDUCER_H_
