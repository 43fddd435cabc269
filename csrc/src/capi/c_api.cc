/*!
 * \file c_api.cc
 * \brief C API (parity: reference `src/c_api.cc`), used by the Python binding.
 *
 * Differences from the reference, by design:
 *  - dispatch keeps dtype/op (AllreduceTyped) so HBM buffers take the RCCL/kernel path;
 *  - long long / unsigned long long are supported (reference c_api.cc:42-84 lacks them);
 *  - checkpoint blobs carry a full uint64 length (reference truncates to uint16 at
 *    c_api.cc:213, corrupting blobs >= 64 KiB);
 *  - checkpoint output buffers are per-thread, not process-global statics;
 *  - an exception never crosses the C boundary: by default it is printed and the process
 *    exits (a failed worker is restarted by the launcher, matching the reference's
 *    die-and-recover model); RabitSetErrorMode(1) makes calls return instead, with the
 *    message in RabitGetLastError().
 */
#include "rabit/c_api.h"

#include <cstdio>
#include <cstring>
#include <string>

#include "coll/host_coll.h"
#include "core/exit.h"
#include "core/trace.h"
#include "device/kernels.h"
#include "engine/engine_base.h"
#include "rabit/internal/io.h"
#include "rabit/rabit.h"

namespace rabit {
namespace engine {
EngineBase *GetEngineBase();
}  // namespace engine
}  // namespace rabit

namespace {
thread_local std::string g_last_error;
int g_error_mode = 0;  // 0: print + exit, 1: record and return

template <typename F>
auto Guard(F &&f, decltype(f()) fallback) -> decltype(f()) {
  try {
    g_last_error.clear();
    return f();
  } catch (const std::exception &e) {
    g_last_error = e.what();
    if (g_error_mode == 0) {
      fprintf(stderr, "xrabit: fatal: %s\n", e.what());
      rabit::utils::ExitProcess(254);
    }
    return fallback;
  }
}

template <typename F>
void GuardVoid(F &&f) {
  Guard([&]() { f(); return 0; }, 0);
}

/*! \brief blob checkpoint: uint64 length + bytes */
struct BlobWriter : public rabit::Serializable {
  const char *data{nullptr};
  size_t length{0};
  void Load(rabit::Stream *) override { rabit::utils::Error("BlobWriter::Load"); }
  void Save(rabit::Stream *fo) const override {
    uint64_t n = length;
    fo->Write(&n, sizeof(n));
    if (n != 0) fo->Write(data, n);
  }
};
struct BlobReader : public rabit::Serializable {
  std::string *out;
  explicit BlobReader(std::string *o) : out(o) {}
  void Load(rabit::Stream *fi) override {
    uint64_t n = 0;
    rabit::utils::Check(fi->Read(&n, sizeof(n)) == sizeof(n), "checkpoint blob: length");
    out->resize(static_cast<size_t>(n));
    if (n != 0) {
      rabit::utils::Check(fi->Read(&(*out)[0], n) == n, "checkpoint blob: payload");
    }
  }
  void Save(rabit::Stream *) const override { rabit::utils::Error("BlobReader::Save"); }
};

rabit::engine::mpi::DataType ToDType(int d) {
  rabit::utils::Check(d >= 0 && d <= 11, "unknown dtype enum %d", d);
  return static_cast<rabit::engine::mpi::DataType>(d);
}
rabit::engine::mpi::OpType ToOp(int o) {
  rabit::utils::Check(o >= 0 && o <= 3, "unknown op enum %d", o);
  return static_cast<rabit::engine::mpi::OpType>(o);
}
}  // namespace

RABIT_DLL bool RabitInit(int argc, char *argv[]) {
  // a process driven through the C API ends on a native error (Guard): a mock kill then ends it
  // at once, like a crash, instead of unwinding the stack first
  rabit::engine::SetMockKillsExit(g_error_mode == 0);
  return Guard([&]() { return rabit::Init(argc, argv); }, false);
}

RABIT_DLL bool RabitFinalize() {
  return Guard([&]() { return rabit::Finalize(); }, false);
}

RABIT_DLL int RabitGetRingPrevRank() {
  return Guard([&]() { return rabit::GetRingPrevRank(); }, -1);
}

RABIT_DLL int RabitGetRank() { return rabit::GetRank(); }

RABIT_DLL int RabitGetWorldSize() { return rabit::GetWorldSize(); }

RABIT_DLL int RabitIsDistributed() { return rabit::IsDistributed() ? 1 : 0; }

RABIT_DLL void RabitTrackerPrint(const char *msg) {
  GuardVoid([&]() { rabit::TrackerPrint(std::string(msg)); });
}

RABIT_DLL void RabitGetProcessorName(char *out_name, rbt_ulong *out_len, rbt_ulong max_len) {
  std::string s = rabit::GetProcessorName();
  if (max_len == 0) {
    *out_len = 0;
    return;
  }
  if (s.length() >= max_len) s.resize(max_len - 1);
  memcpy(out_name, s.c_str(), s.length() + 1);
  *out_len = static_cast<rbt_ulong>(s.length());
}

RABIT_DLL void RabitBroadcast(void *sendrecv_data, rbt_ulong size, int root) {
  GuardVoid([&]() { rabit::Broadcast(sendrecv_data, size, root); });
}

RABIT_DLL void RabitAllgather(void *sendrecvbuf, size_t total_size, size_t beginIndex,
                              size_t size_node_slice, size_t size_prev_slice, int enum_dtype) {
  GuardVoid([&]() {
    const size_t ts = rabit::coll::DTypeSize(ToDType(enum_dtype));
    rabit::engine::GetEngine()->Allgather(sendrecvbuf, total_size * ts, beginIndex * ts,
                                          (beginIndex + size_node_slice) * ts,
                                          size_prev_slice * ts);
  });
}

RABIT_DLL void RabitAllreduce(void *sendrecvbuf, size_t count, int enum_dtype, int enum_op,
                              void (*prepare_fun)(void *arg), void *prepare_arg) {
  GuardVoid([&]() {
    const auto dtype = ToDType(enum_dtype);
    const auto op = ToOp(enum_op);
    if (op == rabit::engine::mpi::kBitwiseOR) {
      rabit::utils::Check(!rabit::engine::mpi::IsFloating(dtype),
                          "BitOR is not defined for floating point types");
    }
    rabit::engine::ReduceFn red = rabit::coll::HostReducer(dtype, op);
    rabit::engine::GetEngine()->AllreduceTyped(sendrecvbuf, count, dtype, op, red, prepare_fun,
                                               prepare_arg);
  });
}

RABIT_DLL int RabitLoadCheckPoint(char **out_global_model, rbt_ulong *out_global_len,
                                  char **out_local_model, rbt_ulong *out_local_len) {
  static thread_local std::string global_buffer, local_buffer;
  return Guard(
      [&]() {
        BlobReader sg(&global_buffer), sl(&local_buffer);
        global_buffer.clear();
        local_buffer.clear();
        int version = rabit::LoadCheckPoint(&sg, out_local_model == nullptr ? nullptr : &sl);
        *out_global_model = rabit::BeginPtr(global_buffer);
        *out_global_len = static_cast<rbt_ulong>(global_buffer.length());
        if (out_local_model != nullptr) {
          *out_local_model = rabit::BeginPtr(local_buffer);
          *out_local_len = static_cast<rbt_ulong>(local_buffer.length());
        }
        return version;
      },
      -1);
}

RABIT_DLL void RabitCheckPoint(const char *global_model, rbt_ulong global_len,
                               const char *local_model, rbt_ulong local_len) {
  GuardVoid([&]() {
    BlobWriter sg, sl;
    sg.data = global_model;
    sg.length = global_len;
    sl.data = local_model;
    sl.length = local_len;
    rabit::CheckPoint(&sg, local_model == nullptr ? nullptr : &sl);
  });
}

RABIT_DLL void RabitLazyCheckPoint(const char *global_model, rbt_ulong global_len) {
  static thread_local BlobWriter lazy;
  GuardVoid([&]() {
    lazy.data = global_model;
    lazy.length = global_len;
    rabit::LazyCheckPoint(&lazy);
  });
}

RABIT_DLL int RabitVersionNumber() { return rabit::VersionNumber(); }

RABIT_DLL int RabitLinkTag() { return 0; }

// ---------------- extensions
RABIT_DLL const char *RabitEngineName() { return rabit::engine::GetEngine()->EngineName(); }

RABIT_DLL void RabitSetStream(void *hip_stream) { rabit::SetStream(hip_stream); }

RABIT_DLL int RabitGetDevice() { return rabit::GetDevice(); }

RABIT_DLL int RabitIsDevicePointer(const void *ptr) { return rabit::IsDevicePointer(ptr) ? 1 : 0; }

RABIT_DLL void RabitSetErrorMode(int mode) {
  g_error_mode = mode;
  rabit::engine::SetMockKillsExit(mode == 0);
}

RABIT_DLL void RabitDevAllreducePrepared(void *dst, const void *src, size_t count,
                                         int enum_dtype, int enum_op, int prep_op,
                                         double alpha) {
  GuardVoid([&]() {
    rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
    rabit::utils::Check(e != nullptr, "device allreduce needs a tracker-backed engine");
    e->DevAllreducePrepared(dst, src, count, ToDType(enum_dtype), ToOp(enum_op), prep_op, alpha,
                            "c_api", 0, "RabitDevAllreducePrepared");
  });
}

RABIT_DLL void *RabitDevSymmetricAlloc(size_t nbytes) {
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  if (e == nullptr || e->device_plane() == nullptr) return nullptr;
  rabit::device::DeviceGuard dg(e->device_plane()->device());
  return e->device_plane()->SymAlloc(nbytes);
}

RABIT_DLL void RabitDevCheckPoint(int n, void *const *ptrs, const size_t *nbytes,
                                  const char *meta, rbt_ulong meta_len) {
  GuardVoid([&]() {
    rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
    rabit::utils::Check(e != nullptr, "device checkpoint needs a tracker-backed engine");
    e->DevCheckPoint(n, ptrs, nbytes, std::string(meta == nullptr ? "" : meta, meta_len));
  });
}

RABIT_DLL void RabitDevCheckPointEx(int n, void *const *ptrs, const size_t *nbytes,
                                    const char *meta, rbt_ulong meta_len, int nl,
                                    void *const *lptrs, const size_t *lnbytes) {
  GuardVoid([&]() {
    rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
    rabit::utils::Check(e != nullptr, "device checkpoint needs a tracker-backed engine");
    e->DevCheckPoint(n, ptrs, nbytes, std::string(meta == nullptr ? "" : meta, meta_len), nl,
                     lptrs, lnbytes);
  });
}

RABIT_DLL int RabitDevLoadCheckPoint(int n, void *const *ptrs, const size_t *nbytes,
                                     char **out_meta, rbt_ulong *out_meta_len) {
  return RabitDevLoadCheckPointEx(n, ptrs, nbytes, out_meta, out_meta_len, 0, nullptr, nullptr);
}

RABIT_DLL int RabitDevLoadCheckPointEx(int n, void *const *ptrs, const size_t *nbytes,
                                       char **out_meta, rbt_ulong *out_meta_len, int nl,
                                       void *const *lptrs, const size_t *lnbytes) {
  static thread_local std::string meta;
  return Guard(
      [&]() {
        rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
        rabit::utils::Check(e != nullptr, "device checkpoint needs a tracker-backed engine");
        meta.clear();
        const int v = e->DevLoadCheckPoint(n, ptrs, nbytes, &meta, nl, lptrs, lnbytes);
        *out_meta = rabit::BeginPtr(meta);
        *out_meta_len = static_cast<rbt_ulong>(meta.size());
        return v;
      },
      -1);
}

RABIT_DLL int RabitDevSetTransport(int which, int direct_mode) {
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  if (e == nullptr || e->device_plane() == nullptr) return -1;
  rabit::device::DevicePlane *d = e->device_plane();
  if (which == 0 && !d->has_comm()) return -1;
  if (which == 1 && !d->has_peers()) return -1;
  if (direct_mode != 0 && !d->has_peers()) return -1;
  if (which < 0 && direct_mode == 0) {
    // back to the calibrated routing: transport and direct form per size band
    d->RestoreCalibrated();
    return 0;
  }
  d->ForceTransport(which);
  if (direct_mode != 0) {
    // 1 pull, 2 push, 3 the pipelined push form
    d->SetDirectPush(direct_mode >= 2);
    d->SetPipeline(direct_mode == 3);
  }
  return 0;
}

RABIT_DLL int RabitDevGraphAllreduce(void *buf, size_t count, int enum_dtype, int enum_op,
                                     void *hip_stream) {
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  if (e == nullptr || e->device_plane() == nullptr) {
    g_last_error = "graph allreduce needs the device plane";
    return -1;
  }
  const char *name = e->EngineName();
  if (!std::strcmp(name, "robust") || !std::strcmp(name, "mock")) {
    // no sequence number, result log or replay: a captured collective cannot be recovered
    g_last_error = "graph allreduce bypasses fault tolerance: use the base engine (lib='base')";
    return -4;
  }
  std::string why;
  const int r = Guard([&]() {
    return e->DevGraphAllreduce(buf, count, enum_dtype, enum_op,
                                static_cast<hipStream_t>(hip_stream), &why);
  }, -1);
  if (r != 0 && !why.empty()) g_last_error = why;
  return r;
}

RABIT_DLL int RabitDevSetFused(int fused) {
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  if (e == nullptr || e->device_plane() == nullptr || !e->device_plane()->has_peers()) return -1;
  e->device_plane()->SetFused(fused != 0);
  return 0;
}

RABIT_DLL int RabitDevSetZeroCopy(size_t min_bytes) {
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  if (e == nullptr || e->device_plane() == nullptr) return -1;
  e->device_plane()->SetZeroCopyMin(min_bytes);
  return 0;
}

RABIT_DLL int RabitDevProbeAllreduce(void *buf, size_t count, int enum_dtype, int enum_op,
                                     int mode) {
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  if (e == nullptr || e->device_plane() == nullptr) return -2;
  return Guard([&]() { return e->DevProbeAllreduce(buf, count, enum_dtype, enum_op, mode); }, -1);
}

RABIT_DLL int RabitDevLinkProbe(size_t nbytes, double *out, int nout) {
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  if (e == nullptr || out == nullptr || nout < rabit::device::PeerGroup::kLinkProbeValues) {
    return -1;
  }
  return Guard([&]() { return e->DevLinkProbe(nbytes, out); }, -1);
}

RABIT_DLL int RabitDevSetPhaseTiming(int on) {
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  if (e == nullptr || e->device_plane() == nullptr) return -1;
  return e->device_plane()->SetPhaseTiming(on != 0) ? 0 : -1;
}

RABIT_DLL const char *RabitGetLastError() { return g_last_error.c_str(); }

RABIT_DLL const char *RabitGetStats() {
  static thread_local std::string stats;
  rabit::engine::EngineBase *e = rabit::engine::GetEngineBase();
  stats = e != nullptr ? e->StatsJson() : std::string("{\"engine\":\"empty\"}");
  return stats.c_str();
}

RABIT_DLL int RabitTraceDump(const char *path) {
  const std::string js = rabit::trace::Tracer::Get().ChromeJson();
  FILE *fp = fopen(path, "w");
  if (fp == nullptr) return -1;
  fwrite(js.data(), 1, js.size(), fp);
  fclose(fp);
  return static_cast<int>(rabit::trace::Tracer::Get().size());
}

RABIT_DLL int RabitDevReduce(void *dst, const void *src, size_t count, int enum_dtype,
                             int enum_op, void *hip_stream) {
  return static_cast<int>(rabit::device::LaunchReduce(dst, src, count, enum_dtype, enum_op,
                                                      static_cast<hipStream_t>(hip_stream)));
}

RABIT_DLL int RabitDevReduceMulti(void *dst, const void *const *srcs, int nsrc, size_t count,
                                  int enum_dtype, int enum_op, void *hip_stream) {
  return static_cast<int>(rabit::device::LaunchReduceMulti(
      dst, srcs, nsrc, count, enum_dtype, enum_op, static_cast<hipStream_t>(hip_stream)));
}

RABIT_DLL int RabitDevPrepare(void *dst, void *dst2, const void *src, size_t count,
                              int enum_dtype, int prep_op, double alpha, void *hip_stream) {
  return static_cast<int>(rabit::device::LaunchPrepare(dst, dst2, src, count, enum_dtype,
                                                       prep_op, alpha,
                                                       static_cast<hipStream_t>(hip_stream)));
}

RABIT_DLL int RabitDevChecksum(const void *buf, size_t nbytes, void *out_dev_u64,
                               void *hip_stream) {
  return static_cast<int>(rabit::device::LaunchChecksum(
      buf, nbytes, static_cast<unsigned long long *>(out_dev_u64),
      static_cast<hipStream_t>(hip_stream)));
}

RABIT_DLL int RabitDevCopy(void *dst, const void *src, size_t nbytes, void *hip_stream) {
  return static_cast<int>(
      rabit::device::LaunchCopy(dst, src, nbytes, static_cast<hipStream_t>(hip_stream)));
}

RABIT_DLL int RabitDevFill(void *dst, size_t count, int enum_dtype, double value,
                           void *hip_stream) {
  return static_cast<int>(rabit::device::LaunchFill(dst, count, enum_dtype, value,
                                                    static_cast<hipStream_t>(hip_stream)));
}
