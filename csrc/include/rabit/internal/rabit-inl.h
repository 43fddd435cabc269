/*!
 * \file rabit-inl.h
 * \brief Template implementation of the public API (parity: reference
 *        `include/rabit/internal/rabit-inl.h:21-383`).
 */
#ifndef RABIT_INTERNAL_RABIT_INL_H_
#define RABIT_INTERNAL_RABIT_INL_H_
#include <cstdarg>
#include <cstring>
#include <functional>
#include <string>
#include <type_traits>
#include <vector>

#include "rabit/internal/engine.h"
#include "rabit/internal/half.h"
#include "rabit/internal/io.h"
#include "rabit/internal/utils.h"

namespace rabit {
namespace engine {
namespace mpi {
/*! \brief C++ type -> dtype enum */
template <typename DType>
inline DataType GetType();
template <> inline DataType GetType<char>() { return kChar; }
template <> inline DataType GetType<signed char>() { return kChar; }
template <> inline DataType GetType<unsigned char>() { return kUChar; }
template <> inline DataType GetType<int>() { return kInt; }
template <> inline DataType GetType<unsigned int>() { return kUInt; }
template <> inline DataType GetType<long>() { return kLong; }                     // NOLINT(*)
template <> inline DataType GetType<unsigned long>() { return kULong; }           // NOLINT(*)
template <> inline DataType GetType<float>() { return kFloat; }
template <> inline DataType GetType<double>() { return kDouble; }
template <> inline DataType GetType<long long>() { return kLongLong; }            // NOLINT(*)
template <> inline DataType GetType<unsigned long long>() { return kULongLong; }  // NOLINT(*)
template <> inline DataType GetType<half_t>() { return kHalf; }
template <> inline DataType GetType<bf16_t>() { return kBFloat16; }
}  // namespace mpi
}  // namespace engine

namespace op {
/*! \brief maximum */
struct Max {
  static const engine::mpi::OpType kType = engine::mpi::kMax;
  template <typename DType>
  inline static void Reduce(DType &dst, const DType &src) {  // NOLINT(*)
    if (src > dst) dst = src;
  }
};
/*! \brief minimum */
struct Min {
  static const engine::mpi::OpType kType = engine::mpi::kMin;
  template <typename DType>
  inline static void Reduce(DType &dst, const DType &src) {  // NOLINT(*)
    if (src < dst) dst = src;
  }
};
/*! \brief sum */
struct Sum {
  static const engine::mpi::OpType kType = engine::mpi::kSum;
  template <typename DType>
  inline static void Reduce(DType &dst, const DType &src) {  // NOLINT(*)
    dst += src;
  }
};
/*! \brief bitwise OR (integer types only) */
struct BitOR {
  static const engine::mpi::OpType kType = engine::mpi::kBitwiseOR;
  template <typename DType>
  inline static void Reduce(DType &dst, const DType &src) {  // NOLINT(*)
    dst |= src;
  }
};
/*! \brief host element-wise reduce function in MPI signature */
template <typename OP, typename DType>
inline void Reducer(const void *src_, void *dst_, int len, const MPI::Datatype &) {
  const DType *__restrict__ src = static_cast<const DType *>(src_);
  DType *__restrict__ dst = static_cast<DType *>(dst_);
  for (int i = 0; i < len; ++i) OP::Reduce(dst[i], src[i]);
}
}  // namespace op

// ---------------- forwarding functions ----------------
inline bool Init(int argc, char *argv[]) { return engine::Init(argc, argv); }
inline bool Finalize() { return engine::Finalize(); }
inline int GetRank() { return engine::GetEngine()->GetRank(); }
inline int GetWorldSize() { return engine::GetEngine()->GetWorldSize(); }
inline bool IsDistributed() { return engine::GetEngine()->IsDistributed(); }
inline std::string GetProcessorName() { return engine::GetEngine()->GetHost(); }
inline int GetRingPrevRank() { return engine::GetEngine()->GetRingPrevRank(); }
inline void SetStream(void *hip_stream) { engine::GetEngine()->SetStream(hip_stream); }
inline int GetDevice() { return engine::GetEngine()->GetDevice(); }
inline bool IsDevicePointer(const void *ptr) { return engine::GetEngine()->IsDevicePointer(ptr); }

inline void Broadcast(void *sendrecv_data, size_t size, int root, const char *_file,
                      const int _line, const char *_caller) {
  engine::GetEngine()->Broadcast(sendrecv_data, size, root, _file, _line, _caller);
}
template <typename DType>
inline void Broadcast(std::vector<DType> *sendrecv_data, int root, const char *_file,
                      const int _line, const char *_caller) {
  static_assert(std::is_trivially_copyable<DType>::value, "Broadcast needs POD element type");
  uint64_t size = sendrecv_data->size();
  Broadcast(&size, sizeof(size), root, _file, _line, _caller);
  if (sendrecv_data->size() != size) sendrecv_data->resize(static_cast<size_t>(size));
  if (size != 0) {
    Broadcast(sendrecv_data->data(), size * sizeof(DType), root, _file, _line, _caller);
  }
}
inline void Broadcast(std::string *sendrecv_data, int root, const char *_file, const int _line,
                      const char *_caller) {
  uint64_t size = sendrecv_data->length();
  Broadcast(&size, sizeof(size), root, _file, _line, _caller);
  if (sendrecv_data->length() != size) sendrecv_data->resize(static_cast<size_t>(size));
  if (size != 0) Broadcast(&(*sendrecv_data)[0], size, root, _file, _line, _caller);
}

template <typename OP, typename DType>
inline void Allreduce(DType *sendrecvbuf, size_t count, void (*prepare_fun)(void *),
                      void *prepare_arg, const char *_file, const int _line,
                      const char *_caller) {
  engine::Allreduce_(sendrecvbuf, sizeof(DType), count, op::Reducer<OP, DType>,
                     engine::mpi::GetType<DType>(), OP::kType, prepare_fun, prepare_arg, _file,
                     _line, _caller);
}

namespace detail {
/*! \brief trampoline that runs a std::function prepare callback */
inline void InvokeLambda(void *fun) { (*static_cast<std::function<void()> *>(fun))(); }
}  // namespace detail

template <typename OP, typename DType>
inline void Allreduce(DType *sendrecvbuf, size_t count, std::function<void()> prepare_fun,
                      const char *_file, const int _line, const char *_caller) {
  engine::Allreduce_(sendrecvbuf, sizeof(DType), count, op::Reducer<OP, DType>,
                     engine::mpi::GetType<DType>(), OP::kType, detail::InvokeLambda,
                     &prepare_fun, _file, _line, _caller);
}

template <typename DType>
inline void Allgather(DType *sendrecvbuf, size_t total_size, size_t slice_begin,
                      size_t size_node_slice, size_t size_prev_slice, const char *_file,
                      const int _line, const char *_caller) {
  engine::GetEngine()->Allgather(sendrecvbuf, total_size * sizeof(DType),
                                 slice_begin * sizeof(DType),
                                 (slice_begin + size_node_slice) * sizeof(DType),
                                 size_prev_slice * sizeof(DType), _file, _line, _caller);
}

inline void TrackerPrint(const std::string &msg) { engine::GetEngine()->TrackerPrint(msg); }
inline void TrackerPrintf(const char *fmt, ...) {
  va_list args;
  va_start(args, fmt);
  std::string msg = utils::VFormat(fmt, args);
  va_end(args);
  TrackerPrint(msg);
}

inline int LoadCheckPoint(Serializable *global_model, Serializable *local_model) {
  return engine::GetEngine()->LoadCheckPoint(global_model, local_model);
}
inline void CheckPoint(const Serializable *global_model, const Serializable *local_model) {
  engine::GetEngine()->CheckPoint(global_model, local_model);
}
inline void LazyCheckPoint(const Serializable *global_model) {
  engine::GetEngine()->LazyCheckPoint(global_model);
}
inline int VersionNumber() { return engine::GetEngine()->VersionNumber(); }

// ---------------- user-defined reducers ----------------
namespace detail {
/*! \brief reduce over naturally aligned structs */
template <typename DType, void (*freduce)(DType &dst, const DType &src)>  // NOLINT(*)
inline void StructReduceAligned(const void *src_, void *dst_, int len, const MPI::Datatype &) {
  const DType *src = static_cast<const DType *>(src_);
  DType *dst = static_cast<DType *>(dst_);
  for (int i = 0; i < len; ++i) freduce(dst[i], src[i]);
}
/*! \brief reduce over structs whose size is not a multiple of their alignment in the wire
 *  buffer: copy out, reduce, copy back (avoids unaligned access) */
template <typename DType, void (*freduce)(DType &dst, const DType &src)>  // NOLINT(*)
inline void StructReduceUnaligned(const void *src_, void *dst_, int len,
                                  const MPI::Datatype &) {
  const char *src = static_cast<const char *>(src_);
  char *dst = static_cast<char *>(dst_);
  for (int i = 0; i < len; ++i) {
    DType a, b;
    std::memcpy(&a, dst + i * sizeof(DType), sizeof(DType));
    std::memcpy(&b, src + i * sizeof(DType), sizeof(DType));
    freduce(a, b);
    std::memcpy(dst + i * sizeof(DType), &a, sizeof(DType));
  }
}
}  // namespace detail

template <typename DType, void (*freduce)(DType &dst, const DType &src)>  // NOLINT(*)
inline Reducer<DType, freduce>::Reducer() {
  // the wire buffers are 8-byte aligned: a struct is safe to address in place when its
  // size keeps every element on its natural alignment
  constexpr bool aligned = (sizeof(DType) % alignof(DType)) == 0 && alignof(DType) <= 8;
  if (aligned) {
    handle_.Init(detail::StructReduceAligned<DType, freduce>, sizeof(DType));
  } else {
    handle_.Init(detail::StructReduceUnaligned<DType, freduce>, sizeof(DType));
  }
}
template <typename DType, void (*freduce)(DType &dst, const DType &src)>  // NOLINT(*)
inline void Reducer<DType, freduce>::Allreduce(DType *sendrecvbuf, size_t count,
                                               void (*prepare_fun)(void *), void *prepare_arg,
                                               const char *_file, const int _line,
                                               const char *_caller) {
  handle_.Allreduce(sendrecvbuf, sizeof(DType), count, prepare_fun, prepare_arg, _file, _line,
                    _caller);
}
template <typename DType, void (*freduce)(DType &dst, const DType &src)>  // NOLINT(*)
inline void Reducer<DType, freduce>::Allreduce(DType *sendrecvbuf, size_t count,
                                               std::function<void()> prepare_fun,
                                               const char *_file, const int _line,
                                               const char *_caller) {
  handle_.Allreduce(sendrecvbuf, sizeof(DType), count, detail::InvokeLambda, &prepare_fun,
                    _file, _line, _caller);
}

namespace detail {
/*! \brief Load/Reduce/Save on each fixed-size slot */
template <typename DType>
inline void SerializeReduceSlots(const void *src_, void *dst_, int len,
                                 const MPI::Datatype &dtype) {
  const size_t nbytes = dtype.type_size;
  const char *src = static_cast<const char *>(src_);
  char *dst = static_cast<char *>(dst_);
  DType tdst, tsrc;
  for (int i = 0; i < len; ++i) {
    utils::MemoryFixSizeBuffer fsrc(const_cast<char *>(src) + i * nbytes, nbytes);
    utils::MemoryFixSizeBuffer fdst(dst + i * nbytes, nbytes);
    tsrc.Load(&fsrc);
    tdst.Load(&fdst);
    tdst.Reduce(tsrc, nbytes);
    fdst.Seek(0);
    tdst.Save(&fdst);
  }
}
/*! \brief prepare step: run the user prepare, then serialize every object into its slot */
template <typename DType>
struct SerializeReduceClosure {
  DType *sendrecvobj;
  size_t max_nbyte, count;
  void (*prepare_fun)(void *arg);
  void *prepare_arg;
  std::string *p_buffer;
  inline void Run() {
    if (prepare_fun != nullptr) prepare_fun(prepare_arg);
    for (size_t i = 0; i < count; ++i) {
      utils::MemoryFixSizeBuffer fs(BeginPtr(*p_buffer) + i * max_nbyte, max_nbyte);
      sendrecvobj[i].Save(&fs);
    }
  }
  inline static void Invoke(void *c) { static_cast<SerializeReduceClosure<DType> *>(c)->Run(); }
};
}  // namespace detail

template <typename DType>
inline SerializeReducer<DType>::SerializeReducer() {
  handle_.Init(detail::SerializeReduceSlots<DType>, sizeof(DType));
}
template <typename DType>
inline void SerializeReducer<DType>::Allreduce(DType *sendrecvobj, size_t max_nbyte,
                                               size_t count, void (*prepare_fun)(void *),
                                               void *prepare_arg, const char *_file,
                                               const int _line, const char *_caller) {
  buffer_.resize(max_nbyte * count);
  detail::SerializeReduceClosure<DType> c;
  c.sendrecvobj = sendrecvobj;
  c.max_nbyte = max_nbyte;
  c.count = count;
  c.prepare_fun = prepare_fun;
  c.prepare_arg = prepare_arg;
  c.p_buffer = &buffer_;
  handle_.Allreduce(BeginPtr(buffer_), max_nbyte, count,
                    detail::SerializeReduceClosure<DType>::Invoke, &c, _file, _line, _caller);
  for (size_t i = 0; i < count; ++i) {
    utils::MemoryFixSizeBuffer fs(BeginPtr(buffer_) + i * max_nbyte, max_nbyte);
    sendrecvobj[i].Load(&fs);
  }
}
template <typename DType>
inline void SerializeReducer<DType>::Allreduce(DType *sendrecvobj, size_t max_nbyte,
                                               size_t count, std::function<void()> prepare_fun,
                                               const char *_file, const int _line,
                                               const char *_caller) {
  this->Allreduce(sendrecvobj, max_nbyte, count, detail::InvokeLambda, &prepare_fun, _file,
                  _line, _caller);
}
}  // namespace rabit
#endif  // RABIT_INTERNAL_RABIT_INL_H_
