/*!
 * \file c_api.h
 * \brief C API of xrabit, ABI compatible with the reference (`include/rabit/c_api.h:24-194`)
 *        plus device extensions (RabitDev..., RabitSet... functions).
 *
 * Pointers handed to RabitAllreduce/RabitBroadcast/RabitAllgather may be host memory or
 * HBM; the engine detects which.
 */
#ifndef RABIT_C_API_H_
#define RABIT_C_API_H_

#ifdef __cplusplus
#define RABIT_EXTERN_C extern "C"
#include <cstddef>
#include <cstdint>
#else
#define RABIT_EXTERN_C
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>
#endif

#define RABIT_DLL RABIT_EXTERN_C __attribute__((visibility("default")))

/*! \brief unsigned long, kept for ABI compatibility */
typedef unsigned long rbt_ulong;  // NOLINT(*)

RABIT_DLL bool RabitInit(int argc, char *argv[]);
RABIT_DLL bool RabitFinalize(void);
RABIT_DLL int RabitGetRingPrevRank(void);
RABIT_DLL int RabitGetRank(void);
RABIT_DLL int RabitGetWorldSize(void);
RABIT_DLL int RabitIsDistributed(void);
RABIT_DLL void RabitTrackerPrint(const char *msg);
RABIT_DLL void RabitGetProcessorName(char *out_name, rbt_ulong *out_len, rbt_ulong max_len);
RABIT_DLL void RabitBroadcast(void *sendrecv_data, rbt_ulong size, int root);
/*! \brief allgather; indices are in elements of enum_dtype */
RABIT_DLL void RabitAllgather(void *sendrecvbuf, size_t total_size, size_t beginIndex,
                              size_t size_node_slice, size_t size_prev_slice, int enum_dtype);
RABIT_DLL void RabitAllreduce(void *sendrecvbuf, size_t count, int enum_dtype, int enum_op,
                              void (*prepare_fun)(void *arg), void *prepare_arg);
/*!
 * \brief load the latest checkpoint; the returned pointers stay valid until the next call
 *        from the same thread.  out_local_model may be NULL.
 */
RABIT_DLL int RabitLoadCheckPoint(char **out_global_model, rbt_ulong *out_global_len,
                                  char **out_local_model, rbt_ulong *out_local_len);
RABIT_DLL void RabitCheckPoint(const char *global_model, rbt_ulong global_len,
                               const char *local_model, rbt_ulong local_len);
/*! \brief lazy checkpoint of a global blob: only the pointer is kept, the caller must keep
 *         the blob alive and unchanged until the next checkpoint (xrabit extension) */
RABIT_DLL void RabitLazyCheckPoint(const char *global_model, rbt_ulong global_len);
RABIT_DLL int RabitVersionNumber(void);
/*! \brief a dummy function used to verify the library was linked */
RABIT_DLL int RabitLinkTag(void);

// ---------------- xrabit extensions ----------------
/*! \brief name of the active engine ("robust", "base", "mock", "empty") */
RABIT_DLL const char *RabitEngineName(void);
/*! \brief JSON: sha256 of the library's sources (csrc/), device code target, compile time */
RABIT_DLL const char *RabitBuildInfo(void);
/*! \brief order device collectives after the given hipStream_t (NULL = null stream) */
RABIT_DLL void RabitSetStream(void *hip_stream);
/*! \brief device ordinal of the engine, -1 if none */
RABIT_DLL int RabitGetDevice(void);
/*! \brief 1 if ptr is device memory */
RABIT_DLL int RabitIsDevicePointer(const void *ptr);
/*!
 * \brief fused "lazy prepare" allreduce for HBM buffers: dst = prep(src) then allreduce(dst).
 *        prep_op: 0 copy, 1 square (g*g), 2 scale by alpha, 3 abs.  The prepare kernel is
 *        skipped when the result is recovered from peers (rabit lazy-prepare semantics).
 */
RABIT_DLL void RabitDevAllreducePrepared(void *dst, const void *src, size_t count,
                                         int enum_dtype, int enum_op, int prep_op,
                                         double alpha);
/*!
 * \brief checkpoint n HBM buffers plus a host metadata blob: HBM snapshot + asynchronous
 *        pinned-host mirror, registered as a lazy global checkpoint (version += 1)
 */
RABIT_DLL void RabitDevCheckPoint(int n, void *const *ptrs, const size_t *nbytes,
                                  const char *meta, rbt_ulong meta_len);
/*! \brief load the latest device checkpoint into n HBM buffers; returns the version (0: none)
 *         and the metadata blob (valid until the next call from this thread) */
RABIT_DLL int RabitDevLoadCheckPoint(int n, void *const *ptrs, const size_t *nbytes,
                                     char **out_meta, rbt_ulong *out_meta_len);
/*!
 * \brief RabitDevCheckPoint plus this rank's local model as nl HBM buffers: kept (with the
 *        replicas of the rabit_local_replica ring predecessors) in HBM and replicated over
 *        xGMI by the robust engine
 */
RABIT_DLL void RabitDevCheckPointEx(int n, void *const *ptrs, const size_t *nbytes,
                                    const char *meta, rbt_ulong meta_len, int nl,
                                    void *const *lptrs, const size_t *lnbytes);
/*! \brief RabitDevLoadCheckPoint that also fills the nl local-model buffers */
RABIT_DLL int RabitDevLoadCheckPointEx(int n, void *const *ptrs, const size_t *nbytes,
                                       char **out_meta, rbt_ulong *out_meta_len, int nl,
                                       void *const *lptrs, const size_t *lnbytes);
/*!
 * \brief allocate nbytes from the engine's symmetric heap (rabit_device_symmetric_heap=<size>):
 *        HBM that the peers map through IPC, so an allreduce input placed there is read in
 *        place by the direct transport (no stage copy).  NULL when unavailable or full; the
 *        memory lives until RabitFinalize.
 */
RABIT_DLL void *RabitDevSymmetricAlloc(size_t nbytes);
/*!
 * \brief benchmarking / diagnosis: route device collectives of this rank over one transport
 *        (which: -1 calibrated choice, 0 RCCL, 1 direct) and pick the direct reduce-scatter
 *        variant (direct_mode: 0 unchanged, 1 pull, 2 push, 3 pipelined push: the push of one
 *        chunk and the gather of an older one share a round).  Every rank must make the same
 *        call between the same collectives.  -1 when the transport is not up.
 */
RABIT_DLL int RabitDevSetTransport(int which, int direct_mode);
/*!
 * \brief form of the direct transport's two-shot allreduce: 1 one fused kernel per chunk
 *        (per-tile hand-offs), 0 the classic stage/barrier/reduce/barrier/gather launches.
 *        Every rank must make the same call between the same collectives.
 * \return 0, or -1 when the direct transport is not up
 */
RABIT_DLL int RabitDevSetFused(int fused);
/*!
 * \brief xrabit extension: in-place RCCL allreduce of a device buffer, enqueued on hip_stream
 *        with no host-side synchronisation, so it can be captured into a hipGraph together with
 *        the step's kernels.  Non-fault-tolerant engines only (base / empty): the op has no
 *        sequence number, result log or replay.
 * \return 0; -1 no device plane, -2 no RCCL communicator, -3 dtype/op RCCL lacks (BitOR),
 *         -4 fault-tolerant engine, -5 RCCL refused the call (RabitGetLastError says which)
 */
RABIT_DLL int RabitDevGraphAllreduce(void *buf, size_t count, int enum_dtype, int enum_op,
                                     void *hip_stream);
/*!
 * \brief xrabit extension: the fault-tolerance tax, measured.  The same device allreduce the
 *        robust engine runs (same transports and routing) but outside its result log and
 *        sequence numbering: a collective every rank calls between the same ops, for
 *        benchmarks.  mode 0: in place, host wait (the base engine's op); 1: into a scratch
 *        slot and buf (the robust engine's dual store), host wait; 2: in place, stream-ordered.
 * \return 0; -1 the op failed (no recovery: a probe); -2 no device plane
 */
/*!
 * \brief xrabit extension: ordinary HBM inputs of at least min_bytes are IPC-registered and
 *        read in place by the direct transport's peers (0: never).  Every rank must make the
 *        same call between the same collectives.  \return 0, -1 without a device plane
 */
RABIT_DLL int RabitDevSetZeroCopy(size_t min_bytes);
RABIT_DLL int RabitDevProbeAllreduce(void *buf, size_t count, int enum_dtype, int enum_op,
                                     int mode);
/*!
 * \brief xrabit extension: per-phase hipEvent timing of the direct transport's classic two-shot
 *        allreduce (stage, barrier, reduce, barrier, gather) from now on, with fresh totals
 *        (on = 1), or off (0); averages appear in RabitGetStats as direct_phase_us.
 * \return 0, or -1 without a direct transport
 */
RABIT_DLL int RabitDevSetPhaseTiming(int on);
/*!
 * \brief xGMI link probe over the direct transport (a collective outside the fault-tolerance
 *        log: every rank calls it between the same ops).  out[0..4] (nout >= 5) receive this
 *        rank's GB/s: one link read, one link write (every rank to rank + k at once, mean over
 *        k), all links read, all links write, all links both directions at once.  0 on success,
 *        -2 without a direct transport (world 1, several hosts), -1 on failure.
 */
RABIT_DLL int RabitDevLinkProbe(size_t nbytes, double *out, int nout);
/*! \brief 0 (default): an error prints and exits the process (the launcher restarts it);
 *         1: an error is recorded (RabitGetLastError) and the call returns */
RABIT_DLL void RabitSetErrorMode(int mode);
/*! \brief last error message of this thread (empty if none) */
RABIT_DLL const char *RabitGetLastError(void);
/*! \brief engine statistics as a JSON string (recoveries, bytes, per-op timing) */
RABIT_DLL const char *RabitGetStats(void);
/*! \brief write the recorded engine spans (rabit_trace=1) as a Chrome trace; returns the span
 *         count or -1 */
RABIT_DLL int RabitTraceDump(const char *path);

// ---------------- device kernel entry points (tests / python ops) ----------------
/*! \brief dst[i] = op(dst[i], src[i]) on device buffers, enqueued on stream */
RABIT_DLL int RabitDevReduce(void *dst, const void *src, size_t count, int enum_dtype,
                             int enum_op, void *hip_stream);
/*! \brief dst[i] = op(srcs[0][i], ..., srcs[nsrc-1][i]) (nsrc <= 8) */
RABIT_DLL int RabitDevReduceMulti(void *dst, const void *const *srcs, int nsrc, size_t count,
                                  int enum_dtype, int enum_op, void *hip_stream);
/*! \brief dst = prep(src) and, if dst2 != NULL, dst2 = prep(src) in the same pass */
RABIT_DLL int RabitDevPrepare(void *dst, void *dst2, const void *src, size_t count,
                              int enum_dtype, int prep_op, double alpha, void *hip_stream);
/*! \brief 64-bit position-weighted checksum of nbytes (nbytes % 4 == 0) into *out (device u64) */
RABIT_DLL int RabitDevChecksum(const void *buf, size_t nbytes, void *out_dev_u64,
                               void *hip_stream);
/*! \brief HBM-to-HBM copy with the gfx950 copy kernel */
RABIT_DLL int RabitDevCopy(void *dst, const void *src, size_t nbytes, void *hip_stream);
/*! \brief fill count elements with value */
RABIT_DLL int RabitDevFill(void *dst, size_t count, int enum_dtype, double value,
                           void *hip_stream);
#endif  // RABIT_C_API_H_
