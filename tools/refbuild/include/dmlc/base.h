/*!
 * \file dmlc/base.h
 * \brief Minimal stand-in for dmlc-core's base.h (not in this image), written only so the
 *        reference rabit sources can be compiled from /root/reference for head-to-head speed
 *        runs (tools/refbuild/build_reference.sh).  Not part of the xrabit library.
 */
#ifndef DMLC_BASE_H_
#define DMLC_BASE_H_
#ifndef DMLC_USE_CXX11
#define DMLC_USE_CXX11 1
#endif
#define DMLC_ENABLE_STD_THREAD 1
#define DMLC_CXX11_THREAD_LOCAL 1
#define DMLC_MODERN_THREAD_LOCAL 1
#define DMLC_THROW_EXCEPTION noexcept(false)
#define DMLC_NO_EXCEPTION noexcept(true)
#endif  // DMLC_BASE_H_
