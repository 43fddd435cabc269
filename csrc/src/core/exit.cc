/*!
 * \file exit.cc
 * \brief ExitProcess: sockets down, exit code to the launcher, _Exit (see exit.h).
 */
#include "core/exit.h"

#include <fcntl.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace rabit {
namespace utils {
namespace {
/*! \brief "fd:inode" (decimal) without sscanf: nothing on this path takes a lock or allocates */
bool ParseFdIno(const char *s, int *fd, unsigned long long *ino) {
  long long f = 0;
  unsigned long long i = 0;
  const char *c = s;
  if (*c < '0' || *c > '9') return false;
  for (; *c >= '0' && *c <= '9'; ++c) f = f * 10 + (*c - '0');
  if (*c++ != ':' || *c < '0' || *c > '9') return false;
  for (; *c >= '0' && *c <= '9'; ++c) i = i * 10 + static_cast<unsigned long long>(*c - '0');
  if (*c != '\0' || f > 1 << 30) return false;
  *fd = static_cast<int>(f);
  *ino = i;
  return true;
}

void ShutdownIfSocket(int fd) {
  struct stat st;
  if (fstat(fd, &st) == 0 && S_ISSOCK(st.st_mode)) (void)shutdown(fd, SHUT_RDWR);
}
}  // namespace

void ExitProcess(int code) {
  fflush(stdout);
  fflush(stderr);
  // every socket, not only rabit's links: the process ends anyway, and a peer or the tracker
  // blocked on any of them should learn it now.  Nothing below allocates (this may run on the
  // watchdog thread while another thread holds the allocator's lock): the descriptors are
  // listed with the raw getdents64 call into a stack buffer.
  const int dir = open("/proc/self/fd", O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (dir >= 0) {
    alignas(8) char buf[4096];
    for (;;) {
      const long got = syscall(SYS_getdents64, dir, buf, sizeof(buf));
      if (got <= 0) break;
      for (long at = 0; at < got;) {
        // struct linux_dirent64: u64 ino, s64 off, u16 reclen, u8 type, char name[]
        unsigned short reclen;
        std::memcpy(&reclen, buf + at + 16, sizeof(reclen));
        const char *name = buf + at + 19;
        if (name[0] >= '0' && name[0] <= '9') {
          int fd = 0;
          for (const char *c = name; *c >= '0' && *c <= '9'; ++c) fd = fd * 10 + (*c - '0');
          if (fd != dir) ShutdownIfSocket(fd);
        }
        at += reclen;
      }
    }
    close(dir);
  } else {
    for (int fd = 3; fd < 4096; ++fd) ShutdownIfSocket(fd);
  }
  // "fd:inode": a process that inherited the variable but not the descriptor (a grandchild
  // started with close_fds) may hold something else under that number; write only to the pipe
  const char *spec = getenv("XRABIT_EXIT_FD");
  int fd = -1;
  unsigned long long ino = 0;
  struct stat st;
  if (spec != nullptr && ParseFdIno(spec, &fd, &ino) && fstat(fd, &st) == 0 &&
      S_ISFIFO(st.st_mode) && static_cast<unsigned long long>(st.st_ino) == ino) {
    char msg[16];
    size_t len = 0;
    unsigned v = code < 0 ? static_cast<unsigned>(-code) : static_cast<unsigned>(code);
    char digits[12];
    size_t nd = 0;
    do {
      digits[nd++] = static_cast<char>('0' + v % 10);
      v /= 10;
    } while (v != 0 && nd < sizeof(digits));
    if (code < 0) msg[len++] = '-';
    while (nd > 0) msg[len++] = digits[--nd];
    msg[len++] = '\n';
    (void)!write(fd, msg, len);
  }
  std::_Exit(code);
}

}  // namespace utils
}  // namespace rabit
