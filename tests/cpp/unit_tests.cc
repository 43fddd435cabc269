/*!
 * \file unit_tests.cc
 * \brief C++ unit tests (own minimal harness; GoogleTest is not available offline).
 *
 * Mirrors the reference's test/cpp suite (test_utils, test_io, allreduce_base_test,
 * allreduce_mock_test, allreduce_robust_test) against xrabit internals, plus serializer,
 * reducer and consensus-encoding tests.  All tests run in single-node mode (no tracker).
 */
#include <rabit/internal/half.h>
#include <rabit/internal/io.h>
#include <rabit/internal/utils.h>
#include <rabit/rabit.h>

#include <atomic>
#include <cmath>
#include <chrono>
#include <cstdio>
#include <functional>
#include <limits>
#include <map>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include "coll/host_coll.h"
#include "core/exit.h"
#include "core/params.h"
#include "core/wait_state.h"
#include "net/link_reset.h"
#include "engine/engine_mock.h"
#include "engine/engine_robust.h"
#include "engine/routing.h"
#include "device/device_plane.h"
#include "device/p2p_plan.h"
#include "device/bcast_plan.h"
#include "device/ar_plan.h"
#include "device/host_stager.h"

namespace {
struct TestCase {
  const char *name;
  std::function<void()> fn;
};
std::vector<TestCase> &Registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Registrar {
  Registrar(const char *name, std::function<void()> fn) { Registry().push_back({name, fn}); }
};
#define TEST(name)                                    \
  void test_##name();                                 \
  Registrar reg_##name(#name, test_##name);           \
  void test_##name()

int g_failures = 0;
#define EXPECT(cond)                                                              \
  do {                                                                            \
    if (!(cond)) {                                                                \
      fprintf(stderr, "  EXPECT failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                               \
    }                                                                             \
  } while (0)
#define EXPECT_THROW(stmt)            \
  do {                                \
    bool thrown = false;              \
    try {                             \
      stmt;                           \
    } catch (const rabit::Error &) {  \
      thrown = true;                  \
    }                                 \
    EXPECT(thrown);                   \
  } while (0)

std::vector<char *> Argv(std::vector<std::string> &store) {
  std::vector<char *> v;
  for (auto &s : store) v.push_back(&s[0]);
  return v;
}

// white-box accessors through inheritance (no #define private public)
class ProbeBase : public rabit::engine::EngineBase {
 public:
  const rabit::net::TrackerConfig &tracker() const { return tracker_; }
  const rabit::coll::HostCollConfig &host() const { return hcfg_; }
  bool bootstrap() const { return bootstrap_cache_; }
  bool debug() const { return debug_; }
  bool timeout() const { return timeout_enabled_; }
  int timeout_sec() const { return timeout_sec_; }
};

class ProbeRobust : public rabit::engine::EngineRobust {
 public:
  using EngineRobust::ActionSummary;
  using EngineRobust::ResultLog;
  static constexpr SeqType kCacheSeq = kCache;
  int result_round() const { return result_buffer_round_; }
};

std::atomic<int> g_timeouts{0};
void CountTimeout(int, int) { g_timeouts.fetch_add(1); }
}  // namespace

// ---------------------------------------------------------------- utils / io
TEST(exit_process_reports_code_and_shuts_sockets) {
  // a child leaving through ExitProcess (csrc/src/core/exit.h): its exit status is the code, a
  // peer on a connected socket sees EOF, and the launcher's pipe gets "77\n" -- only when the
  // XRABIT_EXIT_FD spec names that pipe's inode (a stale spec must write nothing)
  for (int right_inode = 1; right_inode >= 0; --right_inode) {
    int pfd[2], sv[2];
    EXPECT(pipe(pfd) == 0);
    EXPECT(socketpair(AF_UNIX, SOCK_STREAM, 0, sv) == 0);
    struct stat st;
    EXPECT(fstat(pfd[1], &st) == 0);
    char spec[64];
    std::snprintf(spec, sizeof(spec), "%d:%llu", pfd[1],
                  static_cast<unsigned long long>(st.st_ino) + (right_inode ? 0 : 1));
    const pid_t pid = fork();
    if (pid == 0) {
      close(pfd[0]);
      close(sv[1]);
      setenv("XRABIT_EXIT_FD", spec, 1);
      rabit::utils::ExitProcess(77);
    }
    close(pfd[1]);
    close(sv[0]);
    char buf[16] = {0};
    ssize_t got = 0;
    for (ssize_t k; (k = read(pfd[0], buf + got, sizeof(buf) - 1 - got)) > 0;) got += k;
    int status = 0;
    EXPECT(waitpid(pid, &status, 0) == pid);
    EXPECT(WIFEXITED(status) && WEXITSTATUS(status) == 77);
    if (right_inode) {
      EXPECT(got == 3 && std::string(buf) == "77\n");
    } else {
      EXPECT(got == 0);
    }
    char c;
    EXPECT(read(sv[1], &c, 1) == 0);
    close(pfd[0]);
    close(sv[1]);
  }
}

TEST(utils_assert_throws) {
  EXPECT_THROW(rabit::utils::Assert(false, "boom %d", 1));
  EXPECT_THROW(rabit::utils::Check(false, "bad"));
  rabit::utils::Assert(true, "never");
  EXPECT(rabit::utils::StringToBool("true") && rabit::utils::StringToBool("1") &&
         !rabit::utils::StringToBool("0") && !rabit::utils::StringToBool("false"));
}

TEST(io_fixed_buffer_seek_end) {
  std::vector<char> buf(64);
  rabit::utils::MemoryFixSizeBuffer fs(buf.data(), buf.size());
  fs.Seek(rabit::utils::MemoryFixSizeBuffer::SeekEnd);
  EXPECT(fs.Tell() == buf.size());
  fs.Seek(60);
  EXPECT_THROW(fs.Write("12345678", 8));
}

TEST(io_buffer_stream_roundtrip) {
  std::string blob;
  rabit::utils::MemoryBufferStream out(&blob);
  std::vector<float> v = {1.5f, -2.0f, 3.25f};
  std::string s = "hello";
  std::vector<std::string> vs = {"a", "", "ccc"};
  std::map<int, double> m = {{1, 0.5}, {7, 2.0}};
  int x = 42;
  out.Write(v);
  out.Write(s);
  out.Write(vs);
  out.Write(m);
  out.Write(x);
  // dmlc byte format: uint64 count then payload
  uint64_t n0;
  std::memcpy(&n0, blob.data(), 8);
  EXPECT(n0 == 3 && blob.size() >= 8 + 12);
  rabit::utils::MemoryBufferStream in(&blob);
  std::vector<float> v2;
  std::string s2;
  std::vector<std::string> vs2;
  std::map<int, double> m2;
  int x2 = 0;
  EXPECT(in.Read(&v2) && in.Read(&s2) && in.Read(&vs2) && in.Read(&m2) && in.Read(&x2));
  EXPECT(v2 == v && s2 == s && vs2 == vs && m2 == m && x2 == 42);
  EXPECT(!in.Read(&x2));
}

TEST(params_parse_unit) {
  EXPECT(rabit::core::ParseUnit("x", "12") == 12);
  EXPECT(rabit::core::ParseUnit("x", "3K") == 3u << 10);
  EXPECT(rabit::core::ParseUnit("x", "256MB") == 256u << 20);
  EXPECT(rabit::core::ParseUnit("x", "2G") == size_t(2) << 30);
  EXPECT_THROW(rabit::core::ParseUnit("x", "abc"));
  EXPECT_THROW(rabit::core::ParseUnit("x", "3Q"));
}

// ---------------------------------------------------------------- host reducers
TEST(host_reducers) {
  using namespace rabit::engine::mpi;
  std::vector<float> a = {1, 5, 3}, b = {4, 2, 3};
  rabit::coll::HostReducer(kFloat, kMax)(b.data(), a.data(), 3, MPI::Datatype(4));
  EXPECT((a == std::vector<float>{4, 5, 3}));
  std::vector<int64_t> c = {1, 2}, d = {6, 8};
  rabit::coll::HostReducer(kLongLong, kBitwiseOR)(d.data(), c.data(), 2, MPI::Datatype(8));
  EXPECT(c[0] == 7 && c[1] == 10);
  EXPECT(rabit::coll::HostReducer(kDouble, kBitwiseOR) == nullptr);
  std::vector<unsigned char> e = {200, 3}, f = {100, 9};
  rabit::coll::HostReducer(kUChar, kMin)(f.data(), e.data(), 2, MPI::Datatype(1));
  EXPECT(e[0] == 100 && e[1] == 3);
  EXPECT(rabit::coll::DTypeSize(kChar) == 1 && rabit::coll::DTypeSize(kULong) == 8);
}

// ---------------------------------------------------------------- base engine params
TEST(base_params_single_node) {
  std::vector<std::string> args = {"rabit_task_id=7",      "rabit_bootstrap_cache=1",
                                   "rabit_debug=true",     "rabit_reduce_ring_mincount=1",
                                   "rabit_timeout=1",      "rabit_timeout_sec=5",
                                   "rabit_reduce_buffer=1M", "not_a_param"};
  auto argv = Argv(args);
  ProbeBase e;
  EXPECT(e.Init(static_cast<int>(argv.size()), argv.data()));
  EXPECT(e.tracker().task_id == "7");
  EXPECT(e.bootstrap() && e.debug() && e.timeout() && e.timeout_sec() == 5);
  EXPECT(e.host().reduce_ring_mincount == 1);
  EXPECT(e.host().reduce_buffer_bytes == (1u << 20));
  EXPECT(e.GetRank() == 0 && e.GetWorldSize() == 1 && !e.IsDistributed());
  // single node: collectives return after running prepare
  int calls = 0;
  void (*prep)(void *) = [](void *p) { ++*static_cast<int *>(p); };
  int v = 3;
  e.Allreduce(&v, 4, 1, rabit::coll::HostReducer(rabit::engine::mpi::kInt, rabit::engine::mpi::kSum),
              prep, &calls, "f", 1, "c");
  EXPECT(calls == 1 && v == 3);
  EXPECT_THROW(ProbeBase().SetParam("rabit_reduce_ring_mincount", "0"));
  e.Shutdown();
}

// ---------------------------------------------------------------- mock engine
TEST(mock_allreduce_throws) {
  std::vector<std::string> args = {"mock=0,0,0,0"};
  auto argv = Argv(args);
  rabit::engine::EngineMock m;
  m.Init(1, argv.data());
  m.TestSetState(0, 0, 0);
  EXPECT_THROW(m.Allreduce(nullptr, 0, 0, nullptr, nullptr, nullptr, "f", 1, "c"));
}

TEST(mock_broadcast_throws_at_version_seq) {
  std::vector<std::string> args = {"mock=0,1,2,0"};
  auto argv = Argv(args);
  rabit::engine::EngineMock m;
  m.Init(1, argv.data());
  m.TestSetState(0, 1, 2);
  EXPECT_THROW(m.Broadcast(nullptr, 0, 0, "f", 1, "c"));
  // the trial counter moved on: the same key no longer fires
  m.Broadcast(nullptr, 0, 0, "f", 1, "c");
}

TEST(mock_gather_throws) {
  std::vector<std::string> args = {"mock=0,0,0,0"};
  auto argv = Argv(args);
  rabit::engine::EngineMock m;
  m.Init(1, argv.data());
  EXPECT_THROW(m.Allgather(nullptr, 0, 0, 0, 0, "f", 1, "c"));
}

TEST(mock_bad_param) {
  rabit::engine::EngineMock m;
  EXPECT_THROW(m.SetParam("mock", "1,2"));
}

// ---------------------------------------------------------------- robust engine
TEST(robust_result_round) {
  std::vector<std::string> args = {"rabit_global_replica=0"};
  auto argv = Argv(args);
  ProbeRobust r;
  r.Init(1, argv.data());
  EXPECT(r.result_round() == -1);
  r.Shutdown();
}

TEST(consensus_reducer) {
  using AS = ProbeRobust::ActionSummary;
  AS a(AS::kCheckPoint, 1, 5, 3), b(0, 1, 7, 9);
  AS::Reducer(&a, &b, 1, MPI::Datatype(8));
  EXPECT(b.seqno() == 5);
  EXPECT(b.check_point() && b.diff_seq() && !b.load_check());
  EXPECT(b.seqno(ProbeRobust::kCacheSeq) == 9);
  EXPECT(b.flag(ProbeRobust::kCacheSeq) == 1);
  AS c(AS::kLoadCheck, 0, 4, 2), d(0, 1, 4, 2);
  AS::Reducer(&c, &d, 1, MPI::Datatype(8));
  EXPECT(!d.diff_seq() && d.load_check() && d.flag(ProbeRobust::kCacheSeq) == 0);
}

TEST(result_log_host) {
  ProbeRobust::ResultLog log;
  void *p = log.AllocTemp(12, false);
  std::memcpy(p, "abcdefghijk", 12);
  log.PushTemp(0, 12);
  void *q = log.AllocTemp(4, false);
  std::memcpy(q, "xyz", 4);
  log.PushTemp(3, 4);
  EXPECT(log.LastSeqNo() == 3);
  const auto *e = log.Query(0);
  EXPECT(e != nullptr && e->size == 12 && !strcmp(static_cast<char *>(log.Data(*e)), "abcdefghijk"));
  EXPECT(log.Query(1) == nullptr);
  EXPECT_THROW(log.PushTemp(2, 4));
  log.DropLast();
  EXPECT(log.LastSeqNo() == 0);
  log.Clear();
  EXPECT(log.LastSeqNo() == -1 && log.size() == 0);
}

TEST(robust_watchdog_times_out) {
  std::vector<std::string> args = {"rabit_timeout=1", "rabit_timeout_sec=1"};
  auto argv = Argv(args);
  ProbeRobust r;
  r.SetTimeoutHandler(CountTimeout);
  r.Init(2, argv.data());
  g_timeouts = 0;
  EXPECT(!r.TestCheckAndRecover(rabit::net::Status::kSockError));
  std::this_thread::sleep_for(std::chrono::milliseconds(1500));
  EXPECT(g_timeouts.load() == 1 && r.watchdog_fired());
  r.Shutdown();
}

TEST(robust_watchdog_recovered_in_time) {
  std::vector<std::string> args = {"rabit_timeout=1", "rabit_timeout_sec=1"};
  auto argv = Argv(args);
  ProbeRobust r;
  r.SetTimeoutHandler(CountTimeout);
  r.Init(2, argv.data());
  g_timeouts = 0;
  EXPECT(!r.TestCheckAndRecover(rabit::net::Status::kSockError));
  std::this_thread::sleep_for(std::chrono::milliseconds(400));
  EXPECT(r.TestCheckAndRecover(rabit::net::Status::kSuccess));
  std::this_thread::sleep_for(std::chrono::milliseconds(1200));
  EXPECT(g_timeouts.load() == 0 && !r.watchdog_fired());
  r.Shutdown();
}

TEST(robust_watchdog_second_error_keeps_deadline) {
  std::vector<std::string> args = {"rabit_timeout=1", "rabit_timeout_sec=1", "rabit_debug=1"};
  auto argv = Argv(args);
  ProbeRobust r;
  r.SetTimeoutHandler(CountTimeout);
  r.Init(3, argv.data());
  g_timeouts = 0;
  EXPECT(!r.TestCheckAndRecover(rabit::net::Status::kSockError));
  std::this_thread::sleep_for(std::chrono::milliseconds(700));
  EXPECT(!r.TestCheckAndRecover(rabit::net::Status::kConnReset));
  std::this_thread::sleep_for(std::chrono::milliseconds(600));
  // 1.3 s after the first error: the deadline counts from the first failure
  EXPECT(g_timeouts.load() == 1);
  r.Shutdown();
}

TEST(robust_shutdown_before_timeout) {
  std::vector<std::string> args = {"rabit_timeout=1", "rabit_timeout_sec=1"};
  auto argv = Argv(args);
  ProbeRobust r;
  r.SetTimeoutHandler(CountTimeout);
  r.Init(2, argv.data());
  g_timeouts = 0;
  EXPECT(!r.TestCheckAndRecover(rabit::net::Status::kSockError));
  EXPECT(r.Shutdown());
  std::this_thread::sleep_for(std::chrono::milliseconds(1200));
  EXPECT(g_timeouts.load() == 0);
}

TEST(half_types_roundtrip_and_rounding) {
  // every non-NaN binary16 / bfloat16 pattern survives f() -> FromFloat()
  int bad = 0;
  for (uint32_t b = 0; b < 65536; ++b) {
    rabit::half_t h;
    h.bits = static_cast<uint16_t>(b);
    const float f = h.f();
    if (f == f && rabit::half_t(f).bits != h.bits) ++bad;
    rabit::bf16_t g;
    g.bits = static_cast<uint16_t>(b);
    const float fg = g.f();
    if (fg == fg && rabit::bf16_t(fg).bits != g.bits) ++bad;
  }
  EXPECT(bad == 0);
  EXPECT(rabit::half_t(1.0f).bits == 0x3c00);
  EXPECT(rabit::half_t(65504.0f).bits == 0x7bff);
  EXPECT(rabit::half_t(65520.0f).bits == 0x7c00);            // rounds to inf
  EXPECT(rabit::half_t(5.9604645e-08f).bits == 0x0001);      // 2^-24, smallest subnormal
  EXPECT(rabit::half_t(2.9802322e-08f).bits == 0x0000);      // 2^-25 ties to even (zero)
  EXPECT(rabit::half_t(1.0f + 1.0f / 2048).bits == 0x3c00);  // tie -> even
  EXPECT(rabit::half_t(1.0f + 3.0f / 2048).bits == 0x3c02);  // tie -> even (up)
  EXPECT(rabit::bf16_t(1.0f).bits == 0x3f80);
  EXPECT(rabit::bf16_t(1.0f + 1.0f / 256).bits == 0x3f80);   // tie -> even
  EXPECT(rabit::bf16_t(1.0f + 3.0f / 256).bits == 0x3f82);
  const float nan = std::numeric_limits<float>::quiet_NaN();
  EXPECT(rabit::half_t(nan).f() != rabit::half_t(nan).f());
  EXPECT(rabit::bf16_t(nan).f() != rabit::bf16_t(nan).f());
  // the host reducer of the extended enum
  rabit::bf16_t a[3] = {rabit::bf16_t(1.0f), rabit::bf16_t(-2.0f), rabit::bf16_t(3.5f)};
  rabit::bf16_t b[3] = {rabit::bf16_t(2.0f), rabit::bf16_t(5.0f), rabit::bf16_t(-1.0f)};
  rabit::coll::HostReducer(rabit::engine::mpi::kBFloat16, rabit::engine::mpi::kSum)(
      b, a, 3, MPI::Datatype(2));
  EXPECT(a[0].f() == 3.0f && a[1].f() == 3.0f && a[2].f() == 2.5f);
  EXPECT(rabit::coll::HostReducer(rabit::engine::mpi::kHalf, rabit::engine::mpi::kBitwiseOR) ==
         nullptr);
  EXPECT(rabit::coll::DTypeSize(rabit::engine::mpi::kHalf) == 2);
}

// the calibration's RCCL / direct routing (routing.h): 64 KiB and 128 MiB points, times in s
TEST(calibration_routing) {
  using rabit::engine::ChooseDirectRouting;
  const double x0 = 65536, x1 = 134217728, none = static_cast<double>(static_cast<size_t>(-1));
  // direct faster at both points with a flatter slope: direct for every size
  auto r = ChooseDirectRouting(x0, x1, 30e-6, 900e-6, 20e-6, 700e-6);
  EXPECT(r.min_bytes == 0 && r.below_bytes == 0);
  // RCCL faster small, direct faster large: direct from the crossover, which lies in between
  r = ChooseDirectRouting(x0, x1, 20e-6, 900e-6, 40e-6, 700e-6);
  EXPECT(r.min_bytes > x0 && r.min_bytes < x1 && r.below_bytes == 0);
  // the crossover of the two lines: equal predicted times there
  const double br = (900e-6 - 20e-6) / (x1 - x0), bd = (700e-6 - 40e-6) / (x1 - x0);
  const double m = static_cast<double>(r.min_bytes);
  EXPECT(std::abs((20e-6 + br * (m - x0)) - (40e-6 + bd * (m - x0))) < 1e-9);
  // direct faster small, RCCL faster large: direct below the crossover only
  r = ChooseDirectRouting(x0, x1, 40e-6, 700e-6, 20e-6, 900e-6);
  EXPECT(static_cast<double>(r.min_bytes) == none && r.below_bytes > x0 && r.below_bytes < x1);
  // RCCL faster at both points: no direct range
  r = ChooseDirectRouting(x0, x1, 20e-6, 700e-6, 40e-6, 900e-6);
  EXPECT(static_cast<double>(r.min_bytes) == none && r.below_bytes == 0);
  // direct faster at the large point only, but with a steeper slope (cannot happen with a
  // straight line through both points unless it is faster at the small one too): from 0
  r = ChooseDirectRouting(x0, x1, 20e-6, 900e-6, 10e-6, 890e-6);
  EXPECT(r.min_bytes == 0);
}

// the piecewise routing over several calibration points (routing.h: ChooseRoutes)
TEST(calibration_routing_piecewise) {
  using rabit::engine::ChooseRoutes;
  using rabit::engine::RouteFor;
  const double K = 1024, M = 1024 * 1024;
  const std::vector<double> x = {64 * K, 1 * M, 4 * M, 32 * M, 128 * M};
  // candidate 0 ("RCCL"): 30 us floor, 200 GB/s; candidate 1 ("direct"): 15 us, 150 GB/s; so
  // direct below the crossover (~2.4 MB), RCCL above
  auto lin = [](double a, double gbps, double s) { return a + s / (gbps * 1e9); };
  std::vector<std::vector<double>> t(2, std::vector<double>(x.size()));
  for (size_t i = 0; i < x.size(); ++i) {
    t[0][i] = lin(30e-6, 200, x[i]);
    t[1][i] = lin(15e-6, 150, x[i]);
  }
  auto r = ChooseRoutes(x, t);
  EXPECT(r.size() == 2 && r[0].lo == 0 && r[0].choice == 1 && r[1].choice == 0);
  const double cross = 15e-6 / (1 / 150e9 - 1 / 200e9);  // equal times there
  EXPECT(std::abs(r[1].lo - cross) < 1.0);
  EXPECT(RouteFor(r, 64 * K) == 1 && RouteFor(r, 128 * M) == 0 && RouteFor(r, 1e12) == 0);
  // three candidates, two crossovers: 0 wins small, 1 in the middle (4-32 MiB), 2 large
  std::vector<std::vector<double>> u = {{10e-6, 40e-6, 120e-6, 800e-6, 3000e-6},
                                        {20e-6, 45e-6, 100e-6, 600e-6, 2600e-6},
                                        {40e-6, 70e-6, 130e-6, 650e-6, 2000e-6}};
  r = ChooseRoutes(x, u);
  EXPECT(r.size() == 3 && r[0].choice == 0 && r[1].choice == 1 && r[2].choice == 2);
  EXPECT(r[1].lo > 1 * M && r[1].lo < 4 * M && r[2].lo > 32 * M && r[2].lo < 128 * M);
  // every measured point routes to its own fastest candidate
  for (size_t i = 0; i < x.size(); ++i) {
    int best = 0;
    for (int c = 1; c < 3; ++c) best = u[c][i] < u[best][i] ? c : best;
    EXPECT(RouteFor(r, x[i]) == best);
  }
  // a candidate that failed (< 0 everywhere) is never chosen; one measured only at some points
  // competes only between them
  u[0] = {-1, -1, -1, -1, -1};
  r = ChooseRoutes(x, u);
  EXPECT(RouteFor(r, 64 * K) == 1 && RouteFor(r, 128 * M) == 2);
  u[1] = {5e-6, 6e-6, -1, -1, -1};
  r = ChooseRoutes(x, u);
  EXPECT(RouteFor(r, 64 * K) == 1 && RouteFor(r, 512 * K) == 1 && RouteFor(r, 8 * M) == 2);
  // past the last point the last interval's lines extend: a flatter candidate takes over
  std::vector<std::vector<double>> v = {{10e-6, 20e-6, 30e-6, 100e-6, 400e-6},
                                        {50e-6, 55e-6, 60e-6, 120e-6, 410e-6}};
  r = ChooseRoutes(x, v);
  EXPECT(RouteFor(r, 128 * M) == 0 && RouteFor(r, 1024 * M) == 1);
  // one point: one band; no measurement: no bands
  EXPECT(ChooseRoutes({64 * K}, {{3e-6}, {2e-6}}).size() == 1);
  EXPECT(ChooseRoutes({64 * K}, {{3e-6}, {2e-6}})[0].choice == 1);
  EXPECT(ChooseRoutes({64 * K, 1 * M}, {{-1, -1}}).empty());
}

TEST(wait_state_working_vs_waiting) {
  using rabit::core::OpScope;
  using rabit::core::WaitScope;
  using rabit::core::WorkingFor;
  EXPECT(WorkingFor() == 0.0);  // outside any op nothing counts
  {
    WaitScope w;  // a wait outside an op does not start a working stretch
  }
  EXPECT(WorkingFor() == 0.0);
  {
    OpScope op;
    std::this_thread::sleep_for(std::chrono::milliseconds(30));
    EXPECT(WorkingFor() >= 0.025);
    {
      OpScope nested;  // nested ops keep the outer stretch
      EXPECT(WorkingFor() >= 0.025);
      WaitScope w;
      EXPECT(WorkingFor() == 0.0);  // waiting on peers: not working
      {
        WaitScope w2;
      }
      EXPECT(WorkingFor() == 0.0);  // still inside the outer wait
    }
    // the wait ended inside the op: a fresh stretch starts
    EXPECT(WorkingFor() < 0.025);
  }
  EXPECT(WorkingFor() == 0.0);
}

// ---------------------------------------------------------------- public API, single node
namespace {
struct Point {
  double x;
  int n;
};
void AddPoint(Point &dst, const Point &src) {  // NOLINT(*)
  dst.x += src.x;
  dst.n += src.n;
}
struct Packed {
  char c[3];
};
void MaxPacked(Packed &dst, const Packed &src) {  // NOLINT(*)
  for (int i = 0; i < 3; ++i) dst.c[i] = std::max(dst.c[i], src.c[i]);
}
}  // namespace

namespace {
/*! \brief a connected loopback TCP pair */
void LoopbackPair(rabit::net::TcpSocket *a, rabit::net::TcpSocket *b) {
  rabit::net::TcpSocket lis;
  lis.Create();
  const int port = lis.BindListenRange(19500, 20500);
  EXPECT(port > 0);
  a->Create();
  EXPECT(a->Connect("127.0.0.1", port));
  *b = lis.Accept();
}
TEST(watchdog_device_wait_limit_clamp) {
  using rabit::core::EffectiveDeviceWaitLimit;
  EXPECT(EffectiveDeviceWaitLimit(0, 100, 30) == 0);       // watchdog off
  EXPECT(EffectiveDeviceWaitLimit(600, 0, 30) == 600);     // no op deadline: the plain limit
  EXPECT(EffectiveDeviceWaitLimit(600, 60, 30) == 600);    // op deadline well inside the limit
  // an op deadline past the limit (explicit rabit_device_op_timeout, or the auto deadline of a
  // very large op): the rank reaches its own deadline and drains before the watchdog fires
  EXPECT(EffectiveDeviceWaitLimit(600, 900, 30) == 935);
  EXPECT(EffectiveDeviceWaitLimit(600, rabit::device::AutoOpDeadline(size_t(700) << 30), 30) >
         rabit::device::AutoOpDeadline(size_t(700) << 30) + 30);
  {
    rabit::core::DeviceDeadlineScope d(123);
    EXPECT(rabit::core::GlobalWaitState().device_op_deadline.load() == 123);
  }
  EXPECT(rabit::core::GlobalWaitState().device_op_deadline.load() == 0);
}

// ---------------------------------------------------------------- RCCL p2p plans (offline)
// The grouped ncclSend / ncclRecv paths of the device plane only run with two or more GPUs;
// a send whose receive has a different size or order is a hang on the first real run.  These
// tests check the plans device_plane.cc executes, for every rank of n = 2..8.
namespace p2p = rabit::device;

// every send s->d has a receive d<-s of equal bytes, in the same per-pair order
void ExpectPaired(const std::vector<std::vector<p2p::P2POp>> &per_rank) {
  const int n = static_cast<int>(per_rank.size());
  for (int s = 0; s < n; ++s) {
    for (int d = 0; d < n; ++d) {
      if (s == d) continue;
      std::vector<size_t> sends, recvs;
      for (const auto &o : per_rank[s]) {
        if (o.send && o.peer == d) sends.push_back(o.bytes);
      }
      for (const auto &o : per_rank[d]) {
        if (!o.send && o.peer == s) recvs.push_back(o.bytes);
      }
      EXPECT(sends == recvs);
    }
    for (const auto &o : per_rank[s]) EXPECT(o.peer != s && o.peer >= 0 && o.peer < n);
  }
}

TEST(p2p_segment_plan_pairs_and_covers) {
  const size_t counts[] = {0, 1, 7, 255, 256, 257, 1000, 4097, 65536 + 3, 300000 + 17};
  const size_t tns[] = {1, 2, 4, 8, 12};
  for (int n = 2; n <= 8; ++n) {
    for (size_t count : counts) {
      for (size_t tn : tns) {
        const p2p::SegmentPlan plan(count, tn, n);
        // segments tile [0, count) exactly once, in rank order, starts 256-element aligned
        size_t next = 0;
        for (int k = 0; k < n; ++k) {
          EXPECT(plan.lo(k) == next || plan.elems(k) == 0);
          EXPECT(plan.lo(k) % 256 == 0 || plan.lo(k) == count);
          next = std::max(next, plan.hi(k));
        }
        EXPECT(next == count);
        std::vector<std::vector<p2p::P2POp>> scatter(n), gather(n);
        for (int r = 0; r < n; ++r) {
          scatter[r] = plan.ScatterOps(r);
          gather[r] = plan.GatherOps(r);
        }
        ExpectPaired(scatter);
        ExpectPaired(gather);
        for (int r = 0; r < n; ++r) {
          // scatter: rank r sends segment k (bytes of its input at lo(k)) to rank k, and receives
          // its own segment from every other rank into inbox slot `sender`, inside the inbox
          for (const auto &o : scatter[r]) {
            if (o.send) {
              EXPECT(o.buf == p2p::kBufIn && o.offset == plan.lo(o.peer) * tn &&
                     o.bytes == plan.elems(o.peer) * tn);
            } else {
              EXPECT(o.buf == p2p::kBufInbox && o.offset == o.peer * plan.slot_bytes(r) &&
                     o.bytes == plan.elems(r) * tn);
              EXPECT(o.offset + o.bytes <= plan.inbox_bytes(r));
              EXPECT(o.offset % 256 == 0);
            }
          }
          // gather: every byte of the output lands once, at the segment's own offset
          std::vector<int> covered(count * tn, 0);
          for (size_t i = plan.lo(r) * tn; i < plan.hi(r) * tn; ++i) covered[i] += 1;
          for (const auto &o : gather[r]) {
            EXPECT(o.buf == p2p::kBufOut);
            if (o.send) {
              EXPECT(o.offset == plan.lo(r) * tn && o.bytes == plan.elems(r) * tn);
            } else {
              EXPECT(o.offset == plan.lo(o.peer) * tn && o.bytes == plan.elems(o.peer) * tn);
              for (size_t i = o.offset; i < o.offset + o.bytes; ++i) covered[i] += 1;
            }
          }
          bool once = true;
          for (int c : covered) once = once && c == 1;
          EXPECT(once);
          // reduce passes: every rank's copy of segment r is reduced exactly once, the running
          // result leads every pass after the first, at most 8 sources per pass
          std::vector<int> used(n, 0);
          const auto passes = plan.ReducePasses(r, 8);
          EXPECT(passes.empty() == (plan.elems(r) == 0));
          for (size_t p = 0; p < passes.size(); ++p) {
            EXPECT(passes[p].size() <= 8 && !passes[p].empty());
            EXPECT((passes[p][0] == -1) == (p > 0));
            for (int k : passes[p]) {
              if (k >= 0) used[k] += 1;
            }
          }
          if (!passes.empty()) {
            for (int k = 0; k < n; ++k) EXPECT(used[k] == 1);
          }
        }
      }
    }
  }
}

TEST(p2p_reduce_passes_many_sources) {
  // more ranks than sources per pass (the same plan with a small pass width)
  const p2p::SegmentPlan plan(1 << 20, 4, 8);
  const auto passes = plan.ReducePasses(3, 3);
  std::vector<int> order;
  for (const auto &p : passes) {
    for (int k : p) {
      if (k >= 0) order.push_back(k);
    }
  }
  EXPECT(order == std::vector<int>({0, 1, 2, 3, 4, 5, 6, 7}));  // rank order: deterministic sums
  EXPECT(passes.size() == 4);  // 3 + (acc + 2) + (acc + 2) + (acc + 1)
}

TEST(p2p_allgather_pieces_cover_slices) {
  std::mt19937 rng(7);
  for (int n = 2; n <= 8; ++n) {
    for (int trial = 0; trial < 200; ++trial) {
      // rabit's ring layout: slices back to back from a random start, wrapping past the end
      const size_t total = 1 + rng() % 5000;
      std::vector<size_t> begin(n), size(n);
      size_t cut = rng() % total, left = total;
      for (int r = 0; r < n; ++r) {
        size[r] = r + 1 == n ? left : (left == 0 ? 0 : rng() % (left + 1));
        left -= size[r];
        begin[r] = cut;
        cut = (cut + size[r]) % total;
      }
      std::vector<int> owner(total, -1), hits(total, 0);
      for (const auto &p : p2p::AllgatherPieces(total, begin, size)) {
        EXPECT(p.bytes > 0 && p.offset + p.bytes <= total);
        for (size_t i = p.offset; i < p.offset + p.bytes; ++i) {
          hits[i] += 1;
          owner[i] = p.root;
        }
      }
      // every byte comes exactly once, from the rank whose slice holds it
      for (int r = 0; r < n; ++r) {
        for (size_t j = 0; j < size[r]; ++j) EXPECT(owner[(begin[r] + j) % total] == r);
      }
      bool once = true;
      for (int h : hits) once = once && h == 1;
      EXPECT(once);
    }
  }
  const std::vector<size_t> ub = {0, 10, 20}, us = {10, 10, 10};
  EXPECT(p2p::AllgatherUniform(30, ub, us));
  EXPECT(!p2p::AllgatherUniform(31, ub, us));
  const std::vector<size_t> wb = {5, 15, 25};
  EXPECT(!p2p::AllgatherUniform(30, wb, us));
}

TEST(p2p_exchange_ops_pair_in_order) {
  struct Item {
    int src, dst, key;
    size_t bytes;
  };
  std::mt19937 rng(11);
  for (int n = 2; n <= 8; ++n) {
    for (int trial = 0; trial < 100; ++trial) {
      std::vector<Item> plan;
      const int m = 1 + rng() % 24;
      for (int i = 0; i < m; ++i) {
        plan.push_back({static_cast<int>(rng() % n), static_cast<int>(rng() % n), i,
                        (rng() % 4 == 0) ? 0 : 1 + rng() % 100000});
      }
      std::vector<std::vector<p2p::P2POp>> per(n);
      std::vector<std::vector<size_t>> item_of(n);
      size_t locals = 0;
      for (int r = 0; r < n; ++r) {
        std::vector<size_t> local;
        per[r] = p2p::ExchangeOps(plan, r, &item_of[r], &local);
        EXPECT(item_of[r].size() == per[r].size());
        for (size_t i : local) EXPECT(plan[i].src == r && plan[i].dst == r && plan[i].bytes > 0);
        locals += local.size();
      }
      ExpectPaired(per);
      // the k-th send s->d and the k-th receive d<-s serve the same plan item
      for (int s = 0; s < n; ++s) {
        for (int d = 0; d < n; ++d) {
          if (s == d) continue;
          std::vector<size_t> si, ri;
          for (size_t i = 0; i < per[s].size(); ++i) {
            if (per[s][i].send && per[s][i].peer == d) si.push_back(item_of[s][i]);
          }
          for (size_t i = 0; i < per[d].size(); ++i) {
            if (!per[d][i].send && per[d][i].peer == s) ri.push_back(item_of[d][i]);
          }
          EXPECT(si == ri);
        }
      }
      size_t want_local = 0, moved = 0;
      for (const Item &x : plan) {
        if (x.bytes != 0 && x.src == x.dst) want_local += 1;
        if (x.bytes != 0 && x.src != x.dst) moved += 1;
      }
      size_t sends = 0;
      for (int r = 0; r < n; ++r) {
        for (const auto &o : per[r]) sends += o.send ? 1 : 0;
      }
      EXPECT(locals == want_local && sends == moved);
    }
  }
}


// ---------------------------------------------------------------- pipelined direct broadcast
// Simulates every rank's stage buffers (2 parities), user buffer and log slot byte by byte over
// consecutive broadcasts (parity carried from op to op).  Rounds between two barriers form an
// interval in which ranks may run in any order, so: a remote read must see a write made in an
// EARLIER interval, and a write must not share an interval with a remote read of the same byte
// (nor follow one without a barrier in between).
namespace {
struct BcastSim {
  int n;
  size_t stage;
  std::vector<std::vector<std::vector<long long>>> st;  // [rank][parity][byte] tag
  std::vector<std::vector<std::vector<int>>> wint;      // interval of the last write
  std::vector<std::vector<std::vector<int>>> rint;      // latest interval of a remote read
  int interval{0};
  BcastSim(int n_, size_t stage_) : n(n_), stage(stage_) {
    st.assign(n, std::vector<std::vector<long long>>(2, std::vector<long long>(stage, -1)));
    wint.assign(n, std::vector<std::vector<int>>(2, std::vector<int>(stage, -1)));
    rint.assign(n, std::vector<std::vector<int>>(2, std::vector<int>(stage, -1)));
  }
  // one broadcast of `bytes` from `root`; returns false on a hazard or wrong data
  bool Run(size_t bytes, size_t chunk, int root, int *parity, size_t *barriers) {
    const rabit::device::BcastPipeline plan(bytes, chunk, n, root);
    std::vector<std::vector<long long>> user(n, std::vector<long long>(bytes, -1)), log = user;
    std::vector<std::vector<int>> uw(n, std::vector<int>(bytes, 0)), lw = uw;
    for (size_t i = 0; i < bytes; ++i) user[root][i] = static_cast<long long>(i);
    bool ok = true;
    const int base = *parity;
    for (size_t t = 0; t < plan.rounds(); ++t) {
      if (plan.barrier_before(t)) {
        ++interval;
        ++*barriers;
      }
      for (int r = 0; r < n; ++r) {
        for (const auto &c : plan.Round(r, t)) {
          const int p = rabit::device::BcastPipeline::parity(base, c.chunk);
          if (c.off + c.bytes > plan.len(c.chunk) || c.off + c.bytes > stage) return false;
          int nd = (c.to_stage ? 1 : 0) + (c.to_user ? 1 : 0) + (c.to_log ? 1 : 0);
          if (nd == 0 || nd > 2) return false;  // the copy kernel stores at most two places
          for (size_t b = 0; b < c.bytes; ++b) {
            const size_t at = c.chunk * plan.chunk + c.off + b;
            long long v;
            if (c.from < 0) {
              v = user[r][at];
            } else {
              v = st[c.from][p][c.off + b];
              if (c.from != r) {
                if (!(wint[c.from][p][c.off + b] < interval)) ok = false;  // read before barrier
                rint[c.from][p][c.off + b] = std::max(rint[c.from][p][c.off + b], interval);
              }
            }
            if (v != static_cast<long long>(at)) ok = false;  // wrong (or stale) bytes
            if (c.to_stage) {
              // nobody may still be reading the old content in this interval
              if (rint[r][p][c.off + b] >= interval) ok = false;
              st[r][p][c.off + b] = v;
              wint[r][p][c.off + b] = interval;
            }
            if (c.to_user) {
              user[r][at] = v;
              uw[r][at] += 1;
            }
            if (c.to_log) {
              log[r][at] = v;
              lw[r][at] += 1;
            }
          }
        }
      }
    }
    *parity = plan.next_parity(base);
    for (int r = 0; r < n; ++r) {
      for (size_t i = 0; i < bytes; ++i) {
        if (user[r][i] != static_cast<long long>(i) || log[r][i] != static_cast<long long>(i)) ok = false;
        if (lw[r][i] != 1 || uw[r][i] != (r == root ? 0 : 1)) ok = false;  // each byte once
      }
    }
    return ok;
  }
};
}  // namespace

TEST(bcast_pipeline_plan_delivers_without_races) {
  using rabit::device::BcastPipeline;
  std::mt19937 rng(5);
  for (int n = 2; n <= 8; ++n) {
    for (int trial = 0; trial < 40; ++trial) {
      const size_t chunk = 256 + rng() % 3000;
      BcastSim sim(n, chunk);
      int parity = static_cast<int>(rng() % 2);
      size_t barriers = 0;
      // consecutive ops with different roots and sizes: hazards across op boundaries count too
      for (int op = 0; op < 4; ++op) {
        const size_t bytes = 1 + rng() % (6 * chunk);
        const int root = static_cast<int>(rng() % n);
        size_t nb = 0;
        const bool ok = sim.Run(bytes, chunk, root, &parity, &nb);
        EXPECT(ok);
        if (!ok) {
          fprintf(stderr, "  n=%d chunk=%zu bytes=%zu root=%d\n", n, chunk, bytes, root);
          return;
        }
        const BcastPipeline plan(bytes, chunk, n, root);
        // nchunks + 1 barriers (n = 2: the final local copy needs none)
        EXPECT(nb == plan.nchunks + (n > 2 ? 1 : 0));
        barriers += nb;
      }
      EXPECT(barriers > 0);
    }
  }
  EXPECT(BcastPipeline(1000, 100, 1, 0).rounds() == 0);  // one rank: nothing to move
  // automatic chunk: sqrt(S x 4 MiB) in 64 KiB steps, at least 1 MiB, at most a stage
  EXPECT(BcastPipeline::AutoChunk(size_t(1) << 30, 256u << 20) == (64u << 20));
  EXPECT(BcastPipeline::AutoChunk(64u << 20, 256u << 20) == (16u << 20));
  EXPECT(BcastPipeline::AutoChunk(4u << 10, 256u << 20) == (1u << 20));
  EXPECT(BcastPipeline::AutoChunk(size_t(16) << 30, 256u << 20) == (256u << 20));
}

// Pipelined two-shot allreduce (ar_plan.h), simulated element by element over consecutive ops
// (parity carried from op to op).  Every stage element carries a tag (element index, mask of the
// ranks summed into it).  Rules, for accesses by ANY rank (the owner's own reduce included):
// a read must see a write from an EARLIER barrier interval, and a write must not share its
// interval with another access of the same element (nor the op boundary, which has no barrier).
namespace {
struct ArSim {
  int n;
  size_t stage;  // elements per parity
  std::vector<std::vector<std::vector<long long>>> st;  // [rank][parity][elem] tag
  std::vector<std::vector<std::vector<int>>> wint, rint;
  int interval{0};
  ArSim(int n_, size_t stage_) : n(n_), stage(stage_) {
    st.assign(n, std::vector<std::vector<long long>>(2, std::vector<long long>(stage, -1)));
    wint.assign(n, std::vector<std::vector<int>>(2, std::vector<int>(stage, -1)));
    rint = wint;
  }
  static long long Tag(size_t idx, int mask) { return static_cast<long long>(idx) * 256 + mask; }
  bool Read(int owner, int p, size_t e, long long *v) {
    if (e >= stage || !(wint[owner][p][e] < interval)) return false;
    rint[owner][p][e] = std::max(rint[owner][p][e], interval);
    *v = st[owner][p][e];
    return true;
  }
  bool Write(int owner, int p, size_t e, long long v) {
    if (e >= stage || rint[owner][p][e] >= interval || wint[owner][p][e] >= interval) return false;
    st[owner][p][e] = v;
    wint[owner][p][e] = interval;
    return true;
  }
  // one allreduce of `count` elements; false on a hazard or a wrong result
  bool Run(size_t count, size_t chunk, int *parity, size_t *barriers) {
    const rabit::device::ArPipeline plan(count, chunk, n);
    if (plan.stage_bytes(1) > stage) return false;
    const int full = (1 << n) - 1;
    std::vector<std::vector<long long>> out(n, std::vector<long long>(count, -1)), second = out;
    std::vector<std::vector<int>> ow(n, std::vector<int>(count, 0)), sw = ow;
    const int base = *parity;
    bool ok = true;
    for (size_t t = 0; t < plan.rounds() && ok; ++t) {
      for (int r = 0; r < n && ok; ++r) {
        for (const auto &c : plan.Copies(r, t)) {
          const int p = rabit::device::ArPipeline::parity(base, c.chunk);
          for (size_t j = 0; j < c.hi - c.lo && ok; ++j) {
            const size_t at = c.chunk * plan.chunk + c.lo + j;
            if (c.push) {
              ok = Write(c.peer, p, plan.inbox(r) + j, Tag(at, 1 << r));
            } else {
              long long v = -1;
              ok = Read(c.peer, p, plan.result() + j, &v) && v == Tag(at, full);
              out[r][at] = v;
              ow[r][at] += 1;
              if (plan.second_in_gather(c.chunk)) {
                second[r][at] = v;
                sw[r][at] += 1;
              }
            }
          }
        }
        const rabit::device::ArReduce red = plan.Reduce(r, t);
        if (red.any) {
          const int p = rabit::device::ArPipeline::parity(base, red.chunk);
          for (size_t j = 0; j < red.hi - red.lo && ok; ++j) {
            const size_t at = red.chunk * plan.chunk + red.lo + j;
            int mask = 0;
            for (int s = 0; s < n && ok; ++s) {
              long long v = -1;
              ok = Read(r, p, plan.inbox(s) + j, &v) && v == Tag(at, 1 << s);
              mask |= 1 << s;
            }
            ok = ok && Write(r, p, plan.result() + j, Tag(at, mask));
          }
        }
      }
      if (plan.barrier_after(t)) {
        ++interval;
        ++*barriers;
      }
    }
    // the guarded tail copy after the last round
    for (int r = 0; r < n; ++r) {
      for (size_t i = 0; i < plan.second_tail(); ++i) {
        second[r][i] = out[r][i];
        sw[r][i] += 1;
      }
    }
    *parity = plan.next_parity(base);
    for (int r = 0; r < n && ok; ++r) {
      for (size_t i = 0; i < count; ++i) {
        if (out[r][i] != Tag(i, full) || second[r][i] != Tag(i, full)) ok = false;
        if (ow[r][i] != 1 || sw[r][i] != 1) ok = false;
      }
    }
    return ok;
  }
};
}  // namespace

TEST(allreduce_pipeline_plan_reduces_without_races) {
  using rabit::device::ArPipeline;
  std::mt19937 rng(9);
  for (int n = 2; n <= 8; ++n) {
    for (int trial = 0; trial < 30; ++trial) {
      const size_t chunk = 256 * static_cast<size_t>(n) * (1 + rng() % 4);
      const ArPipeline probe(chunk, chunk, n);
      ArSim sim(n, probe.stage_bytes(1));
      int parity = static_cast<int>(rng() % 2);
      size_t barriers = 0;
      // consecutive ops of different sizes: hazards across op boundaries count too
      for (int op = 0; op < 3; ++op) {
        const size_t count = 1 + rng() % (chunk * 5);
        size_t nb = 0;
        const bool ok = sim.Run(count, chunk, &parity, &nb);
        EXPECT(ok);
        if (!ok) {
          fprintf(stderr, "  n=%d chunk=%zu count=%zu op=%d\n", n, chunk, count, op);
          return;
        }
        const ArPipeline plan(count, chunk, n);
        EXPECT(nb == plan.nchunks + 1);  // one barrier per round but the last
        barriers += nb;
      }
      EXPECT(barriers > 0);
    }
  }
  // automatic chunk: sqrt(S x 4 MiB), >= 1 MiB, a multiple of 256 n elements, within the stage
  const size_t c128 = ArPipeline::AutoChunk((128u << 20) / 4, 4, 8, 256u << 20);
  EXPECT(c128 % (256 * 8) == 0 && c128 * 4 >= (22u << 20) && c128 * 4 <= (24u << 20));
  EXPECT(ArPipeline(c128, c128, 8).stage_bytes(4) <= (256u << 20));
  const size_t cbig = ArPipeline::AutoChunk(size_t(4) << 30, 4, 8, 256u << 20);
  EXPECT(ArPipeline(cbig, cbig, 8).stage_bytes(4) <= (256u << 20));
  EXPECT(ArPipeline::AutoChunk(1024, 4, 2, 256u << 20) == (1u << 20) / 4);
}

TEST(copy_pool_splits_copies) {
  // the host side of the pipelined host staging: one memcpy split over a pool of threads
  std::mt19937 rng(3);
  for (int threads : {1, 2, 5}) {
    rabit::device::CopyPool pool(threads);
    EXPECT(pool.threads() == threads);
    for (size_t n : {size_t(0), size_t(1), size_t(4097), size_t(1) << 20, (size_t(3) << 20) + 77,
                     (size_t(17) << 20) + 5}) {
      std::vector<unsigned char> src(n + 3), dst(n + 3, 0xee);
      for (auto &c : src) c = static_cast<unsigned char>(rng());
      pool.Copy(dst.data() + 1, src.data() + 2, n);  // unaligned on both sides
      EXPECT(std::equal(src.begin() + 2, src.begin() + 2 + n, dst.begin() + 1));
      EXPECT(dst[0] == 0xee && dst[n + 1] == 0xee);  // nothing outside the range
    }
  }
  EXPECT(rabit::device::CopyPool::AutoThreads() >= 1 && rabit::device::CopyPool::AutoThreads() <= 8);
}

TEST(copy_pool_back_to_back_jobs) {
  // jobs follow each other with no gap, alternating sizes and buffers: a helper that wakes late
  // for one job must neither copy with its pointers into the next nor count a piece of it twice
  // (either would let Copy return before every byte of its job has landed)
  rabit::device::CopyPool pool(6);
  std::mt19937 rng(11);
  std::vector<std::vector<unsigned char>> src(3), dst(3);
  const size_t sizes[3] = {(size_t(1) << 20) + 4096, (size_t(5) << 20) + 3, size_t(2) << 20};
  for (int b = 0; b < 3; ++b) {
    src[b].resize(sizes[b]);
    dst[b].resize(sizes[b]);
  }
  bool ok = true;
  for (int it = 0; it < 300 && ok; ++it) {
    const int b = it % 3;
    const unsigned char v = static_cast<unsigned char>(rng());
    std::fill(src[b].begin(), src[b].end(), v);
    pool.Copy(dst[b].data(), src[b].data(), sizes[b]);
    ok = std::all_of(dst[b].begin(), dst[b].end(), [v](unsigned char c) { return c == v; });
  }
  EXPECT(ok);
}

TEST(rccl_result_classes) {
  using rabit::device::ClassifyRccl;
  using rabit::device::RcclOutcome;
  EXPECT(ClassifyRccl(0) == RcclOutcome::kOk);
  EXPECT(ClassifyRccl(7) == RcclOutcome::kPending);
  // what a dead or aborted peer produces: recoverable
  for (int r : {1, 2, 3, 6}) EXPECT(ClassifyRccl(r) == RcclOutcome::kPeerFailure);
  // usage errors of this library: fatal
  for (int r : {4, 5, 8, 42}) EXPECT(ClassifyRccl(r) == RcclOutcome::kFatal);
}

}  // namespace

TEST(link_reset_discards_stale_bytes) {
  // reference TryResetLinks (allreduce_robust.cc:567-679): stale bytes in both directions are
  // dropped, the stream is usable afterwards
  rabit::net::TcpSocket a, b;
  LoopbackPair(&a, &b);
  std::vector<char> junk_a(200000, 'x'), junk_b(50000, 'y');
  EXPECT(a.SendAll(junk_a.data(), junk_a.size()) == junk_a.size());
  EXPECT(b.SendAll(junk_b.data(), junk_b.size()) == junk_b.size());
  std::vector<rabit::net::TcpSocket *> la = {&a}, lb = {&b};
  rabit::net::Status ra = rabit::net::Status::kSockError, rb = ra;
  // a generous deadline: under ThreadSanitizer on a loaded machine a side can be descheduled for
  // seconds (a passing run takes milliseconds)
  std::thread t([&]() { rb = rabit::net::ResetLinks(lb, 20000); });
  ra = rabit::net::ResetLinks(la, 20000);
  t.join();
  EXPECT(ra == rabit::net::Status::kSuccess && rb == rabit::net::Status::kSuccess);
  a.SetNonBlock(false);
  b.SetNonBlock(false);
  EXPECT(a.SendAll("hello", 5) == 5);
  char got[6] = {0};
  EXPECT(b.RecvAll(got, 5) == 5 && std::string(got) == "hello");
  EXPECT(b.SendAll("world", 5) == 5);
  EXPECT(a.RecvAll(got, 5) == 5 && std::string(got) == "world");
}

TEST(link_reset_dead_peer_fails) {
  rabit::net::TcpSocket a, b;
  LoopbackPair(&a, &b);
  b.Close();
  std::vector<rabit::net::TcpSocket *> la = {&a};
  const auto t0 = std::chrono::steady_clock::now();
  EXPECT(rabit::net::ResetLinks(la, 3000) == rabit::net::Status::kSockError);
  EXPECT(a.IsClosed());
  EXPECT(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(3));
}

TEST(link_reset_silent_peer_times_out) {
  rabit::net::TcpSocket a, b;
  LoopbackPair(&a, &b);  // b never takes part
  std::vector<rabit::net::TcpSocket *> la = {&a};
  EXPECT(rabit::net::ResetLinks(la, 300) == rabit::net::Status::kSockError);
}

TEST(api_uninitialised_single_node) {
  EXPECT(rabit::GetWorldSize() == 1 && rabit::GetRank() == 0);
  std::vector<double> v = {1, 2};
  rabit::Allreduce<rabit::op::Sum>(v.data(), v.size());
  EXPECT(v[1] == 2);
  rabit::Reducer<Point, AddPoint> red;
  Point p[2] = {{1.0, 1}, {2.0, 2}};
  red.Allreduce(p, 2);
  EXPECT(p[1].n == 2);
  rabit::Reducer<Packed, MaxPacked> red2;
  Packed q[1] = {{{1, 2, 3}}};
  red2.Allreduce(q, 1, [&]() { q[0].c[0] = 9; });
  EXPECT(q[0].c[0] == 9);
  std::string s = "abc";
  rabit::Broadcast(&s, 0);
  EXPECT(s == "abc");
}

int main(int argc, char **argv) {
  int failed_cases = 0;
  for (auto &t : Registry()) {
    if (argc > 1 && std::string(argv[1]) != t.name) continue;
    const int before = g_failures;
    try {
      t.fn();
    } catch (const std::exception &e) {
      fprintf(stderr, "  unexpected exception: %s\n", e.what());
      ++g_failures;
    }
    const bool ok = g_failures == before;
    failed_cases += ok ? 0 : 1;
    printf("[%s] %s\n", ok ? "  OK  " : " FAIL ", t.name);
  }
  printf("%zu tests, %d failed\n", Registry().size(), failed_cases);
  return failed_cases == 0 ? 0 : 1;
}
