/*!
 * \file registry.cc
 * \brief Engine selection and the per-thread engine singleton.
 *
 * Parity: reference `src/engine.cc:19-140` (thread-local engine, Init/Finalize/GetEngine,
 * Allgather, Allreduce_, ReduceHandle).  The reference picks the engine at link time; here
 * the library default is a compile-time macro (one .so per flavour, same names as the
 * reference: librabit = robust, librabit_base, librabit_mock, librabit_empty) and the
 * `rabit_engine=robust|base|mock|empty` parameter overrides it at run time.
 * Unlike the reference, Allreduce_ keeps the dtype/op enums (AllreduceTyped) so device
 * buffers can use RCCL and the CDNA4 kernels.
 */
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "coll/host_coll.h"
#include "engine/engine_base.h"
#include "engine/engine_empty.h"
#include "engine/engine_mock.h"
#include "engine/engine_robust.h"
#include "rabit/internal/engine.h"
#include "rabit/internal/utils.h"

#ifndef XRABIT_DEFAULT_ENGINE
#define XRABIT_DEFAULT_ENGINE "robust"
#endif

namespace rabit {
namespace engine {
namespace {
std::atomic<bool> g_mock_kills_exit{false};
}  // namespace
void SetMockKillsExit(bool v) { g_mock_kills_exit.store(v); }
bool MockKillsExit() { return g_mock_kills_exit.load(); }

void IEngine::AllreduceTyped(void *buf, size_t count, mpi::DataType dtype, mpi::OpType op,
                             ReduceFunction reducer, PreprocFunction prepare_fun,
                             void *prepare_arg, const char *_file, const int _line,
                             const char *_caller) {
  (void)op;
  this->Allreduce(buf, coll::DTypeSize(dtype), count, reducer, prepare_fun, prepare_arg, _file,
                  _line, _caller);
}

void IEngine::AllreduceDevice(void *buf, size_t type_nbytes, size_t count,
                              DeviceReduceLauncher *dev_reducer, ReduceFunction host_reducer,
                              PreprocFunction prepare_fun, void *prepare_arg, const char *_file,
                              const int _line, const char *_caller) {
  (void)dev_reducer;
  this->Allreduce(buf, type_nbytes, count, host_reducer, prepare_fun, prepare_arg, _file, _line,
                  _caller);
}

namespace {
struct ThreadEntry {
  std::unique_ptr<IEngine> engine;
  EngineBase *base{nullptr};     // non-null for tracker-backed engines
  EngineEmpty *empty{nullptr};   // non-null for the empty engine
  bool initialized{false};
};

ThreadEntry &Entry() {
  static thread_local ThreadEntry e;
  return e;
}

/*! \brief engine kind: argv rabit_engine=..., then env rabit_engine, then the default */
std::string ChooseEngine(int argc, char *argv[]) {
  std::string kind = XRABIT_DEFAULT_ENGINE;
  const char *env = getenv("rabit_engine");
  if (env != nullptr) kind = env;
  for (int i = 0; i < argc; ++i) {
    if (argv[i] != nullptr && strncmp(argv[i], "rabit_engine=", 13) == 0) kind = argv[i] + 13;
  }
  return kind;
}
}  // namespace

bool Init(int argc, char *argv[]) {
  ThreadEntry &e = Entry();
  if (e.initialized) return true;
  const std::string kind = ChooseEngine(argc, argv);
  bool ok;
  if (kind == "empty") {
    e.empty = new EngineEmpty();
    e.engine.reset(e.empty);
    ok = e.empty->Init(argc, argv);
  } else {
    if (kind == "robust") {
      e.base = new EngineRobust();
    } else if (kind == "mock") {
      e.base = new EngineMock();
    } else if (kind == "base") {
      e.base = new EngineBase();
    } else {
      utils::Error("unknown rabit_engine \"%s\" (robust, base, mock, empty)", kind.c_str());
    }
    e.engine.reset(e.base);
    ok = e.base->Init(argc, argv);
  }
  e.initialized = ok;
  if (!ok) {
    e.engine.reset();
    e.base = nullptr;
    e.empty = nullptr;
  }
  return ok;
}

bool Finalize() {
  ThreadEntry &e = Entry();
  if (!e.initialized) return true;
  bool ok = e.base != nullptr ? e.base->Shutdown() : e.empty->Shutdown();
  e.engine.reset();
  e.base = nullptr;
  e.empty = nullptr;
  e.initialized = false;
  return ok;
}

IEngine *GetEngine() {
  ThreadEntry &e = Entry();
  if (e.initialized) return e.engine.get();
  // not initialised: behave as a single process (reference engine.cc:71-82)
  static thread_local EngineBase single;
  return &single;
}

/*! \brief the engine as EngineBase, or nullptr (empty engine) — used by the C API */
EngineBase *GetEngineBase() {
  ThreadEntry &e = Entry();
  if (e.initialized) return e.base;
  return static_cast<EngineBase *>(GetEngine());
}

void Allgather(void *sendrecvbuf, size_t total_size, size_t slice_begin, size_t slice_end,
               size_t size_prev_slice, const char *_file, const int _line,
               const char *_caller) {
  GetEngine()->Allgather(sendrecvbuf, total_size, slice_begin, slice_end, size_prev_slice, _file,
                         _line, _caller);
}

void Allreduce_(void *sendrecvbuf, size_t type_nbytes, size_t count, IEngine::ReduceFunction red,
                mpi::DataType dtype, mpi::OpType op, IEngine::PreprocFunction prepare_fun,
                void *prepare_arg, const char *_file, const int _line, const char *_caller) {
  (void)type_nbytes;
  GetEngine()->AllreduceTyped(sendrecvbuf, count, dtype, op, red, prepare_fun, prepare_arg,
                              _file, _line, _caller);
}

ReduceHandle::ReduceHandle()
    : handle_(nullptr), redfunc_(nullptr), htype_(nullptr), created_type_nbytes_(0) {}
ReduceHandle::~ReduceHandle() = default;

void ReduceHandle::Init(IEngine::ReduceFunction redfunc, size_t type_nbytes) {
  utils::Assert(redfunc_ == nullptr, "ReduceHandle: can only Init once");
  redfunc_ = redfunc;
  created_type_nbytes_ = type_nbytes;
}

void ReduceHandle::Allreduce(void *sendrecvbuf, size_t type_nbytes, size_t count,
                             IEngine::PreprocFunction prepare_fun, void *prepare_arg,
                             const char *_file, const int _line, const char *_caller) {
  utils::Assert(redfunc_ != nullptr, "ReduceHandle: Init must be called first");
  GetEngine()->Allreduce(sendrecvbuf, type_nbytes, count, redfunc_, prepare_fun, prepare_arg,
                         _file, _line, _caller);
}

int ReduceHandle::TypeSize(const MPI::Datatype &dtype) {
  return static_cast<int>(dtype.type_size);
}
}  // namespace engine
}  // namespace rabit
