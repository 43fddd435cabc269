/*!
 * \file exit.h
 * \brief Leaving the process on a failure the process itself noticed (a native fatal error, a
 *        mock kill, a hang, a wedged device): make the death visible at once, then _Exit.
 *
 * Ending a process that holds GPU memory takes the kernel ~0.2 s: its address space, with every
 * device mapping, is torn down before its file table, so peers see its sockets close -- and the
 * launcher sees it exit -- only at the end of that.  Both waits sat on the survivors' recovery
 * path (profiles/r4_recovery/).  ExitProcess therefore
 *  1. shuts down every socket of the process (the peers' reads and the tracker see EOF now);
 *  2. writes the exit code to the launcher's exit pipe, when the launcher passed one
 *     (XRABIT_EXIT_FD, rabit_amd/launcher.py), so the replacement starts while the kernel is
 *     still tearing this process down;
 *  3. _Exits (no unwinding, no atexit handlers: as a crash would).
 * A process killed from outside (SIGKILL, the OOM killer) is still seen the slow way.
 */
#ifndef XRABIT_CORE_EXIT_H_
#define XRABIT_CORE_EXIT_H_

namespace rabit {
namespace utils {

[[noreturn]] void ExitProcess(int code);

}  // namespace utils
}  // namespace rabit
#endif  // XRABIT_CORE_EXIT_H_
