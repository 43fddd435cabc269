/*!
 * \file thread_local.h
 * \brief ThreadLocalStore<T>::Get(): one lazily built T per calling thread, destroyed when the
 *        thread exits (API of the reference's include/rabit/internal/thread_local.h:38-85).
 *        The reference keeps a registry of heap objects for pre-C++11 compilers; here the
 *        object is a function-local `thread_local`, so there is nothing to register or free.
 */
#ifndef RABIT_INTERNAL_THREAD_LOCAL_H_
#define RABIT_INTERNAL_THREAD_LOCAL_H_

namespace rabit {
template <typename T>
struct ThreadLocalStore {
  /*! \brief this thread's instance (constructed on first use) */
  static T *Get() { return &Slot(); }

 private:
  static T &Slot() {
    thread_local T value{};
    return value;
  }
};
}  // namespace rabit
#endif  // RABIT_INTERNAL_THREAD_LOCAL_H_
