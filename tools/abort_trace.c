// abort_trace.c -- test tooling: a native backtrace on SIGABRT / SIGSEGV / SIGBUS, also after the
// Python interpreter has finalized (faulthandler is off by then, and a crash in a runtime's exit-time
// teardown leaves no other trace).  Loaded with ctypes by tools/run_gpu_suite.py; never by the product.
//   gcc -O1 -g -shared -fPIC tools/abort_trace.c -o tools/libabort_trace.so
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fatal(int sig) {
    static const char hdr[] = "\n[abort_trace] fatal signal, native backtrace:\n";
    ssize_t w = write(2, hdr, sizeof(hdr) - 1);
    (void)w;
    void* frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

__attribute__((constructor)) static void install(void) {
    void* warm[1];
    backtrace(warm, 1);  // loads libgcc_s now, not inside the handler
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_fatal;
    sa.sa_flags = SA_RESETHAND;
    sigaction(SIGABRT, &sa, 0);
    sigaction(SIGSEGV, &sa, 0);
    sigaction(SIGBUS, &sa, 0);
}
