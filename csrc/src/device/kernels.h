/*!
 * \file kernels.h
 * \brief Host-side launchers of the gfx950 HIP kernels of the device data plane.
 *
 * Kernel inventory: K1-K4 element-wise reduce (max/min/sum/bitor, 10
 * dtypes), multi-source reduce (the local step of the all-to-all based allreduce used for
 * ops RCCL lacks, e.g. BitOR), K8 fused lazy-prepare (g*g etc., optionally dual-store),
 * and a position-weighted checksum used to validate recovered buffers and checkpoints.
 * dtype codes are rabit::engine::mpi::DataType; op codes are mpi::OpType.
 */
#ifndef XRABIT_DEVICE_KERNELS_H_
#define XRABIT_DEVICE_KERNELS_H_

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>

namespace rabit {
namespace device {

/*! \brief prepare ops of the fused lazy-prepare kernel */
enum PrepOp : int { kPrepCopy = 0, kPrepSquare = 1, kPrepScale = 2, kPrepAbs = 3 };
constexpr int kMaxReduceSources = 8;

/*! \brief dst[i] = op(dst[i], src[i]) */
hipError_t LaunchReduce(void *dst, const void *src, size_t count, int dtype, int op,
                        hipStream_t stream);
/*!
 * \brief dst[i] = op(srcs[0][i], ..., srcs[nsrc-1][i]), 1 <= nsrc <= 8 (dst may alias any
 *        source).  guard: optional device word; the launch does nothing when it is non-zero
 *        (set by a failed peer barrier earlier on the stream).  table: optional device array of
 *        nsrc source pointers written by an earlier kernel (srcs then only serve the host-side
 *        alignment check and must be aligned like the table's pointers).  post_scale != 0
 *        multiplies the reduced value (float/double only): the averaging of a data-parallel
 *        gradient applied once after the sum, so the inputs can be read unmodified.
 *        dst2: optional second destination written with the same values by the same kernel
 *        (the user buffer next to the result log: one launch and one read instead of two).
 */
/*!
 *        prep != kPrepCopy: the lazy prepare (g*g, alpha*g, |g|) is applied to sources
 *        prep_from..nsrc-1 as they are loaded (the running result of an earlier pass sits at
 *        index 0 with prep_from = 1), so a prepared allreduce needs no pass of its own.
 */
hipError_t LaunchReduceMulti(void *dst, const void *const *srcs, int nsrc, size_t count,
                             int dtype, int op, hipStream_t stream, const int *guard = nullptr,
                             const void *const *table = nullptr, double post_scale = 0.0,
                             void *dst2 = nullptr, int prep = 0, double prep_alpha = 1.0,
                             int prep_from = 0);
/*! \brief dst[i] = prep(src[i]); also dst2[i] when dst2 != nullptr */
hipError_t LaunchPrepare(void *dst, void *dst2, const void *src, size_t count, int dtype,
                         int prep, double alpha, hipStream_t stream);
/*!
 * \brief position-weighted checksum over 16-byte vectors v = (w0, w1, w2, w3) of 32-bit words:
 *        out[0] += sum of all words, out[1] += sum_v (v+1) * (w0 + 2 w1 + 3 w2 + 4 w3)
 *        (mod 2^64); nbytes must be a multiple of 16; out must be zeroed by the caller
 */
hipError_t LaunchChecksum(const void *buf, size_t nbytes, unsigned long long *out,
                          hipStream_t stream);
/*! \brief device-to-device copy: 16-byte-per-lane kernel for the aligned bulk (the blit
 *  kernel behind hipMemcpyAsync D2D streams slower), hipMemcpyAsync for an unaligned rest */
hipError_t LaunchCopy(void *dst, const void *src, size_t bytes, hipStream_t stream);
/*! \brief copy with `ctas` grid-stride workgroups (device -> pinned host mirrors: PCIe-bound,
 *  so a few workgroups suffice and the other CUs stay with the caller's work); dst may be
 *  device-accessible host memory */
hipError_t LaunchCopyNarrow(void *dst, const void *src, size_t bytes, int ctas,
                            hipStream_t stream);
/*!
 * \brief fault injection (mock_dev_hang): a one-wave kernel that models a wedged kernel on the
 *        stream.  It ignores the engine's abort word; it ends when the host sets *release or
 *        after max_ticks of the device wall clock, so no wave outlives the process.
 */
hipError_t LaunchHang(const volatile int *release, long long max_ticks, hipStream_t stream);
/*! \brief fill count elements with value (bit pattern of dtype) */
hipError_t LaunchFill(void *dst, size_t count, int dtype, double value, hipStream_t stream);
}  // namespace device
}  // namespace rabit
#endif  // XRABIT_DEVICE_KERNELS_H_
