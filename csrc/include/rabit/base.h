/*!
 * \file base.h
 * \brief Common definitions.  The reference only carries MSVC CRT macros here
 *        (`include/rabit/base.h:12-17`); xrabit targets Linux/ROCm only.
 */
#ifndef RABIT_BASE_H_
#define RABIT_BASE_H_
#include <cstddef>
#include <cstdint>

#define XRABIT_VERSION_MAJOR 0
#define XRABIT_VERSION_MINOR 1

#endif  // RABIT_BASE_H_
