/* Test helper (not product): on SIGSEGV / SIGBUS / SIGABRT, print the native backtrace with each frame's
 * library and file offset (symbolise later with llvm-symbolizer --obj=<lib> <offset>), then hand the
 * signal to the previous handler (pytest's faulthandler prints the Python stack).
 * Build: gcc -O1 -g -shared -fPIC tests/segv/segv_bt.c -o tests/segv/libsegv_bt.so -ldl
 * Use:   ctypes.CDLL("tests/segv/libsegv_bt.so").segv_bt_install() */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_old[32];

static void handler(int sig, siginfo_t* si, void* uc) {
    void* bt[64];
    const int n = backtrace(bt, 64);
    dprintf(2, "\n[segv_bt] signal %d at address %p; native backtrace (%d frames):\n", sig, si ? si->si_addr : 0, n);
    for (int i = 0; i < n; i++) {
        Dl_info d;
        memset(&d, 0, sizeof(d));
        if (dladdr(bt[i], &d) && d.dli_fname)
            dprintf(2, "[segv_bt]  #%-2d %s +0x%lx  (%s)\n", i, d.dli_fname,
                    (unsigned long)((char*)bt[i] - (char*)d.dli_fbase), d.dli_sname ? d.dli_sname : "?");
        else
            dprintf(2, "[segv_bt]  #%-2d %p\n", i, bt[i]);
    }
    sigaction(sig, &g_old[sig], NULL);
    if (g_old[sig].sa_flags & SA_SIGINFO) {
        if (g_old[sig].sa_sigaction) g_old[sig].sa_sigaction(sig, si, uc);
    } else if (g_old[sig].sa_handler != SIG_IGN && g_old[sig].sa_handler != SIG_DFL && g_old[sig].sa_handler) {
        g_old[sig].sa_handler(sig);
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

int segv_bt_install(void) {
    void* warm[2];
    backtrace(warm, 2); /* load libgcc's unwinder now, not inside the handler */
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    const int sigs[] = {SIGSEGV, SIGBUS, SIGABRT};
    for (unsigned i = 0; i < sizeof(sigs) / sizeof(sigs[0]); i++)
        if (sigaction(sigs[i], &sa, &g_old[sigs[i]]) != 0) return -1;
    return 0;
}
