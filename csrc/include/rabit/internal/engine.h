/*!
 * \file engine.h
 * \brief Engine interface of xrabit.
 *
 * Source-compatible with the reference interface (`include/rabit/internal/engine.h:32-343`):
 * IEngine virtuals, engine::Init/Finalize/GetEngine, Allgather, Allreduce_, mpi::OpType,
 * mpi::DataType and ReduceHandle keep their names and signatures.
 *
 * MI355X extensions (new):
 *  - `IEngine::AllreduceTyped` receives the dtype/op enums (the reference drops them at
 *    `src/engine.cc:98-111`), so a device buffer can be reduced by RCCL or by our own
 *    CDNA4 kernels instead of a host function pointer;
 *  - every collective accepts HBM pointers (hipMalloc / torch CUDA tensors); the engine
 *    detects the pointer kind and routes to the device data plane;
 *  - `SetStream` orders device collectives after the caller's HIP stream.
 */
#ifndef RABIT_INTERNAL_ENGINE_H_
#define RABIT_INTERNAL_ENGINE_H_
#include <string>

#include "rabit/serializable.h"

#ifndef RABIT_API_CALLER_SIGNATURE
#define RABIT_API_CALLER_SIGNATURE
#if defined(__GNUC__) || defined(__clang__)
#define _FILE __builtin_FILE()
#define _LINE __builtin_LINE()
#define _CALLER __builtin_FUNCTION()
#else
#define _FILE "N/A"
#define _LINE -1
#define _CALLER "N/A"
#endif
#endif  // RABIT_API_CALLER_SIGNATURE

namespace MPI {
/*! \brief MPI-compatible datatype handle: carries the element size in bytes */
class Datatype {
 public:
  size_t type_size;
  explicit Datatype(size_t type_size) : type_size(type_size) {}
};
}  // namespace MPI

namespace rabit {
namespace engine {
/*! \brief stubs compatible with MPI */
namespace mpi {
enum OpType { kMax = 0, kMin = 1, kSum = 2, kBitwiseOR = 3 };
enum DataType {
  kChar = 0,
  kUChar = 1,
  kInt = 2,
  kUInt = 3,
  kLong = 4,
  kULong = 5,
  kFloat = 6,
  kDouble = 7,
  kLongLong = 8,
  kULongLong = 9,
  // extensions (no reference equivalent): 16-bit floats, rabit/internal/half.h
  kHalf = 10,
  kBFloat16 = 11
};
/*! \brief floating-point dtypes (BitOR is undefined for them) */
inline bool IsFloating(int d) {
  return d == kFloat || d == kDouble || d == kHalf || d == kBFloat16;
}
}  // namespace mpi

/*! \brief interface of an Allreduce engine */
class IEngine {
 public:
  /*! \brief lazy preprocessing hook, runs before the collective unless the result is recovered */
  typedef void(PreprocFunction)(void *arg);
  /*! \brief MPI-style reduce function; buffers are 8-byte aligned */
  typedef void(ReduceFunction)(const void *src, void *dst, int count, const MPI::Datatype &dtype);

  /*!
   * \brief launcher of a user-defined device reduction (rabit/device_reducer.h):
   *        dst[i] = reduce(srcs[0][i], ..., srcs[nsrc-1][i]) for count elements, enqueued on the
   *        HIP stream `stream`; when guard is non-null the kernel must do nothing if *guard != 0
   *        at its start (a failed peer barrier).  dst may alias srcs[0].  Returns a hipError_t.
   */
  typedef int(DeviceReduceLauncher)(void *dst, const void *const *srcs, int nsrc, size_t count,
                                    const int *guard, void *stream);

  virtual ~IEngine() = default;
  /*! \brief ring allgather: this rank owns [slice_begin, slice_end) of a ring buffer of
   *  total_size bytes; the slice of rank+1 starts at slice_end */
  virtual void Allgather(void *sendrecvbuf, size_t total_size, size_t slice_begin,
                         size_t slice_end, size_t size_prev_slice, const char *_file = _FILE,
                         const int _line = _LINE, const char *_caller = _CALLER) = 0;
  /*! \brief in-place allreduce with an opaque reducer */
  virtual void Allreduce(void *sendrecvbuf_, size_t type_nbytes, size_t count,
                         ReduceFunction reducer, PreprocFunction prepare_fun = nullptr,
                         void *prepare_arg = nullptr, const char *_file = _FILE,
                         const int _line = _LINE, const char *_caller = _CALLER) = 0;
  /*! \brief in-place allreduce of a built-in (dtype, op); host or device buffer.
   *  Default implementation falls back to the opaque-reducer path. */
  virtual void AllreduceTyped(void *sendrecvbuf_, size_t count, mpi::DataType dtype,
                              mpi::OpType op, ReduceFunction reducer,
                              PreprocFunction prepare_fun = nullptr, void *prepare_arg = nullptr,
                              const char *_file = _FILE, const int _line = _LINE,
                              const char *_caller = _CALLER);
  /*!
   * \brief in-place allreduce with a user reduction that has a device form: HBM buffers are
   *        reduced by dev_reducer kernels on the device plane, host buffers by host_reducer.
   *        Default implementation: host_reducer through Allreduce.
   */
  virtual void AllreduceDevice(void *sendrecvbuf_, size_t type_nbytes, size_t count,
                               DeviceReduceLauncher *dev_reducer, ReduceFunction host_reducer,
                               PreprocFunction prepare_fun = nullptr, void *prepare_arg = nullptr,
                               const char *_file = _FILE, const int _line = _LINE,
                               const char *_caller = _CALLER);
  /*! \brief broadcast size bytes from root */
  virtual void Broadcast(void *sendrecvbuf_, size_t size, int root, const char *_file = _FILE,
                         const int _line = _LINE, const char *_caller = _CALLER) = 0;
  /*! \brief reset state after an exception (tests only) */
  virtual void InitAfterException() = 0;
  /*! \brief load the latest checkpoint, returns its version (0 = fresh start) */
  virtual int LoadCheckPoint(Serializable *global_model, Serializable *local_model = nullptr) = 0;
  /*! \brief checkpoint: a stage of execution is finished, version += 1 */
  virtual void CheckPoint(const Serializable *global_model,
                          const Serializable *local_model = nullptr) = 0;
  /*! \brief checkpoint that only remembers the pointer (global model must stay unchanged
   *  until the last collective of this version completes) */
  virtual void LazyCheckPoint(const Serializable *global_model) = 0;
  virtual int VersionNumber() const = 0;
  virtual int GetRingPrevRank() const = 0;
  virtual int GetRank() const = 0;
  virtual int GetWorldSize() const = 0;
  virtual bool IsDistributed() const = 0;
  virtual std::string GetHost() const = 0;
  virtual void TrackerPrint(const std::string &msg) = 0;
  // ---------------- xrabit extensions ----------------
  /*! \brief HIP stream (hipStream_t) that device collectives are ordered after;
   *  nullptr = null stream */
  virtual void SetStream(void *stream) { (void)stream; }
  /*! \brief HIP device ordinal used by this engine, -1 when there is no device plane */
  virtual int GetDevice() const { return -1; }
  /*! \brief true if ptr is device (HBM) memory visible to this engine */
  virtual bool IsDevicePointer(const void *ptr) const { (void)ptr; return false; }
  /*! \brief name of the engine implementation ("robust", "base", "mock", "empty") */
  virtual const char *EngineName() const = 0;
};

/*! \brief initializes the engine of this thread */
bool Init(int argc, char *argv[]);
/*! \brief finalizes the engine of this thread */
bool Finalize();
/*! \brief engine of this thread (an uninitialised single-node engine if Init was not called) */
IEngine *GetEngine();

/*! \brief ring allgather (see IEngine::Allgather) */
void Allgather(void *sendrecvbuf, size_t total_size, size_t slice_begin, size_t slice_end,
               size_t size_prev_slice, const char *_file = _FILE, const int _line = _LINE,
               const char *_caller = _CALLER);
/*! \brief internal typed allreduce used by rabit::Allreduce<OP> */
void Allreduce_(void *sendrecvbuf, size_t type_nbytes, size_t count, IEngine::ReduceFunction red,
                mpi::DataType dtype, mpi::OpType op, IEngine::PreprocFunction prepare_fun = nullptr,
                void *prepare_arg = nullptr, const char *_file = _FILE, const int _line = _LINE,
                const char *_caller = _CALLER);

/*! \brief handle for user-defined reducers (MPI compatibility) */
class ReduceHandle {
 public:
  ReduceHandle();
  ~ReduceHandle();
  /*! \brief set the (commutative) reduce function and the element size */
  void Init(IEngine::ReduceFunction redfunc, size_t type_nbytes);
  void Allreduce(void *sendrecvbuf, size_t type_nbytes, size_t count,
                 IEngine::PreprocFunction prepare_fun = nullptr, void *prepare_arg = nullptr,
                 const char *_file = _FILE, const int _line = _LINE,
                 const char *_caller = _CALLER);
  /*! \return the number of bytes of the type */
  static int TypeSize(const MPI::Datatype &dtype);

 protected:
  void *handle_;
  IEngine::ReduceFunction *redfunc_;
  void *htype_;
  size_t created_type_nbytes_;
};
}  // namespace engine
}  // namespace rabit
#endif  // RABIT_INTERNAL_ENGINE_H_
