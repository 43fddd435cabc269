/*!
 * \file rabit.h
 * \brief xrabit public C++ API: Reliable Allreduce and Broadcast Interface, MI355X-native.
 *
 * Source compatible with the reference API (`include/rabit/rabit.h:94-456`): code written
 * against rabit compiles unchanged.  Buffers may live in host memory or in HBM (hipMalloc,
 * torch CUDA tensors); device buffers are reduced over RCCL/xGMI and CDNA4 HIP kernels.
 *
 * Usage:
 *   rabit::Init(argc, argv);
 *   int iter = rabit::LoadCheckPoint(&model);
 *   for (int i = iter; i < n; ++i) { ...; rabit::Allreduce<rabit::op::Sum>(g, n); ...;
 *                                    rabit::CheckPoint(&model); }
 *   rabit::Finalize();
 */
#ifndef RABIT_RABIT_H_  // NOLINT(*)
#define RABIT_RABIT_H_  // NOLINT(*)
#include <functional>
#include <string>
#include <vector>

#include "rabit/internal/engine.h"
#include "rabit/serializable.h"

namespace rabit {
/*! \brief reduction operators */
namespace op {
struct Max;
struct Min;
struct Sum;
struct BitOR;
}  // namespace op

/*! \brief initialize the engine; argv entries of the form name=value are parameters */
inline bool Init(int argc, char *argv[]);
/*! \brief finalize the engine, call once after all jobs */
inline bool Finalize();
/*! \brief rank of this process */
inline int GetRank();
/*! \brief number of processes */
inline int GetWorldSize();
/*! \brief whether running distributed (a tracker is attached) */
inline bool IsDistributed();
/*! \brief host name of this process */
inline std::string GetProcessorName();
/*! \brief rank of the previous node on the ring */
inline int GetRingPrevRank();
/*! \brief print a message on the tracker */
inline void TrackerPrint(const std::string &msg);
/*! \brief printf-style TrackerPrint */
inline void TrackerPrintf(const char *fmt, ...);
/*! \brief broadcast a memory region (host or HBM) from root */
inline void Broadcast(void *sendrecv_data, size_t size, int root, const char *_file = _FILE,
                      const int _line = _LINE, const char *_caller = _CALLER);
/*! \brief broadcast a std::vector (size first, then payload) */
template <typename DType>
inline void Broadcast(std::vector<DType> *sendrecv_data, int root, const char *_file = _FILE,
                      const int _line = _LINE, const char *_caller = _CALLER);
/*! \brief broadcast a std::string (size first, then payload) */
inline void Broadcast(std::string *sendrecv_data, int root, const char *_file = _FILE,
                      const int _line = _LINE, const char *_caller = _CALLER);
/*!
 * \brief in-place allreduce of count elements of DType with operator OP
 * \param prepare_fun lazy preprocessing called before the reduction unless the result
 *        can be recovered from peers (then it is NOT called)
 */
template <typename OP, typename DType>
inline void Allreduce(DType *sendrecvbuf, size_t count, void (*prepare_fun)(void *) = nullptr,
                      void *prepare_arg = nullptr, const char *_file = _FILE,
                      const int _line = _LINE, const char *_caller = _CALLER);
/*! \brief allreduce with a lambda prepare function */
template <typename OP, typename DType>
inline void Allreduce(DType *sendrecvbuf, size_t count, std::function<void()> prepare_fun,
                      const char *_file = _FILE, const int _line = _LINE,
                      const char *_caller = _CALLER);
/*!
 * \brief ring allgather; all sizes count elements of DType.  This rank owns
 *        [slice_begin, slice_begin + size_node_slice); the slice of rank+1 starts where it
 *        ends (wrapping).  The 4th argument is a SIZE, as in the reference's implementation
 *        (include/rabit/internal/rabit-inl.h:202-213, used so by test/model_recover.cc:82);
 *        the reference's header comment calls it slice_end.
 */
template <typename DType>
inline void Allgather(DType *sendrecvbuf_, size_t total_size, size_t slice_begin,
                      size_t size_node_slice, size_t size_prev_slice, const char *_file = _FILE,
                      const int _line = _LINE, const char *_caller = _CALLER);
/*!
 * \brief load the latest checkpoint
 * \return version of the loaded model; 0 means nothing was checkpointed (models untouched)
 */
inline int LoadCheckPoint(Serializable *global_model, Serializable *local_model = nullptr);
/*! \brief checkpoint the models; version number increases by one */
inline void CheckPoint(const Serializable *global_model,
                       const Serializable *local_model = nullptr);
/*! \brief lazy checkpoint of the global model (pointer only, serialized on demand) */
inline void LazyCheckPoint(const Serializable *global_model);
/*! \brief number of checkpoints taken so far */
inline int VersionNumber();
// ---------------- MI355X extensions ----------------
/*! \brief order device collectives after this HIP stream (hipStream_t); nullptr = null stream */
inline void SetStream(void *hip_stream);
/*! \brief HIP device used by the engine (-1: no device plane) */
inline int GetDevice();
/*! \brief true if ptr points into HBM of the engine's device */
inline bool IsDevicePointer(const void *ptr);

namespace engine {
class ReduceHandle;
}  // namespace engine

/*!
 * \brief user-defined reducer over a struct type; freduce(dst, src) must be commutative.
 *        Device buffers are staged through host memory for this reducer.
 */
template <typename DType, void (*freduce)(DType &dst, const DType &src)>  // NOLINT(*)
class Reducer {
 public:
  Reducer();
  inline void Allreduce(DType *sendrecvbuf, size_t count, void (*prepare_fun)(void *) = nullptr,
                        void *prepare_arg = nullptr, const char *_file = _FILE,
                        const int _line = _LINE, const char *_caller = _CALLER);
  inline void Allreduce(DType *sendrecvbuf, size_t count, std::function<void()> prepare_fun,
                        const char *_file = _FILE, const int _line = _LINE,
                        const char *_caller = _CALLER);

 private:
  engine::ReduceHandle handle_;
};

/*!
 * \brief reducer for variable-size objects serialized into fixed max_nbyte slots.
 *        DType must provide Load(Stream*), Save(Stream*) const and Reduce(const DType&, size_t
 * max_nbyte).
 */
template <typename DType>
class SerializeReducer {
 public:
  SerializeReducer();
  inline void Allreduce(DType *sendrecvobj, size_t max_nbyte, size_t count,
                        void (*prepare_fun)(void *) = nullptr, void *prepare_arg = nullptr,
                        const char *_file = _FILE, const int _line = _LINE,
                        const char *_caller = _CALLER);
  inline void Allreduce(DType *sendrecvobj, size_t max_nbyte, size_t count,
                        std::function<void()> prepare_fun, const char *_file = _FILE,
                        const int _line = _LINE, const char *_caller = _CALLER);

 private:
  engine::ReduceHandle handle_;
  std::string buffer_;
};
}  // namespace rabit
#include "rabit/internal/rabit-inl.h"
#endif  // RABIT_RABIT_H_ // NOLINT(*)
