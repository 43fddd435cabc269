/*!
 * \file exit.cc
 * \brief ExitProcess: sockets down, exit code to the launcher, _Exit (see exit.h).
 */
#include "core/exit.h"

#include <dirent.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace rabit {
namespace utils {
namespace {
void ShutdownIfSocket(int fd) {
  struct stat st;
  if (fstat(fd, &st) == 0 && S_ISSOCK(st.st_mode)) (void)shutdown(fd, SHUT_RDWR);
}
}  // namespace

void ExitProcess(int code) {
  fflush(stdout);
  fflush(stderr);
  // every socket, not only rabit's links: the process ends anyway, and a peer or the tracker
  // blocked on any of them should learn it now
  DIR *d = opendir("/proc/self/fd");
  if (d != nullptr) {
    const int self = dirfd(d);
    while (struct dirent *e = readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      const int fd = atoi(e->d_name);
      if (fd != self) ShutdownIfSocket(fd);
    }
    closedir(d);
  } else {
    for (int fd = 3; fd < 4096; ++fd) ShutdownIfSocket(fd);
  }
  // "fd:inode": a process that inherited the variable but not the descriptor (a grandchild
  // started with close_fds) may hold something else under that number; write only to the pipe
  const char *spec = getenv("XRABIT_EXIT_FD");
  int fd = -1;
  unsigned long long ino = 0;
  struct stat st;
  if (spec != nullptr && sscanf(spec, "%d:%llu", &fd, &ino) == 2 && fd >= 0 &&
      fstat(fd, &st) == 0 && S_ISFIFO(st.st_mode) &&
      static_cast<unsigned long long>(st.st_ino) == ino) {
    char msg[16];
    const int len = snprintf(msg, sizeof(msg), "%d\n", code);
    (void)!write(fd, msg, static_cast<size_t>(len));
  }
  std::_Exit(code);
}

}  // namespace utils
}  // namespace rabit
