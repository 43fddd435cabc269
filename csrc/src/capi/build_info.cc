/*!
 * \file build_info.cc
 * \brief What a library was built from: a hash of every source under csrc/ (computed by the
 *        Makefile when this file is compiled) and the device code target.  rabit_amd._lib
 *        compares the hash with the working tree, so a test (CPU and GPU box alike) can tell a
 *        library that matches its sources from a stale one.
 */
#include "rabit/c_api.h"

#ifndef XRABIT_SRC_HASH
#define XRABIT_SRC_HASH "unknown"
#endif
#ifndef XRABIT_ARCH
#define XRABIT_ARCH "unknown"
#endif

RABIT_DLL const char *RabitBuildInfo() {
  return "{\"src_sha256\":\"" XRABIT_SRC_HASH "\",\"offload_arch\":\"" XRABIT_ARCH
         "\",\"compiled\":\"" __DATE__ " " __TIME__ "\"}";
}
