/* Debug helper (not product code): load with ctypes before a run to print the native
 * backtrace of a host SIGSEGV; resolve the "lib.so(+0x...)" frames with addr2line. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void on_segv(int sig, siginfo_t *si, void *ctx) {
    (void)ctx;
    void *bt[64];
    char msg[128];
    int n = snprintf(msg, sizeof msg, "segv_trace: signal %d at address %p\n", sig, si->si_addr);
    write(2, msg, n);
    int k = backtrace(bt, 64);
    backtrace_symbols_fd(bt, k, 2);
    _exit(128 + sig);
}

__attribute__((constructor)) static void install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, NULL);
    sigaction(SIGBUS, &sa, NULL);
}
