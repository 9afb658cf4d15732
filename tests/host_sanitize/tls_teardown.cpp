// Thread-teardown marker of the fake HIP runtime, TEST INFRASTRUCTURE ONLY
// (hip/hip_runtime.h fakehip::tls_teardown).
//
// The C++ runtime registers each thread_local destructor through glibc's
// __cxa_thread_atexit_impl, and a thread runs them in reverse order of
// registration.  This definition (the harness executable's, found before
// glibc's) registers the destructor, then registers the marker after it: the
// marker is always the thread's most recent registration, so it runs before
// every thread_local destructor of the thread and flags the thread as in
// teardown.  From then on each fake HIP entry point aborts — whatever order
// the real runtime's or a profiler's thread-local state would have been torn
// down in, a HIP call from a thread_local destructor is caught.
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>

#include <hip/hip_runtime.h>

namespace {

using AtExit = int (*)(void (*)(void*), void*, void*);

AtExit real_atexit() {
  static const AtExit f = reinterpret_cast<AtExit>(dlsym(RTLD_NEXT, "__cxa_thread_atexit_impl"));
  if (!f) {
    std::fprintf(stderr, "tls_teardown: no __cxa_thread_atexit_impl to wrap\n");
    std::abort();
  }
  return f;
}

void mark_teardown(void*) { fakehip::tls_teardown() = true; }

}  // namespace

extern "C" int __cxa_thread_atexit_impl(void (*dtor)(void*), void* obj, void* dso) {
  const int rc = real_atexit()(dtor, obj, dso);
  if (rc == 0 && dtor != &mark_teardown) (void)real_atexit()(&mark_teardown, nullptr, dso);
  return rc;
}
