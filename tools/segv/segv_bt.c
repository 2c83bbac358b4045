/* Test-only diagnostic: on SIGSEGV print the native backtrace of the faulting
 * thread to stderr, then hand the signal to the previously installed handler
 * (Python's faulthandler, which prints the Python frames).  fd: where to
 * write (pytest captures fd 2, so tests pass a file of their own).  Loaded by
 * tests/conftest.py when MOE_SEGV_BT=1; host code only. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static struct sigaction g_prev;
static int g_fd = 2;

static void on_segv(int sig, siginfo_t* info, void* uc) {
  void* frames[64];
  const char msg[] = "\n[segv_bt] native backtrace:\n";
  if (write(g_fd, msg, sizeof(msg) - 1) < 0) { /* nothing to do */ }
  int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, g_fd);
  sigaction(SIGSEGV, &g_prev, NULL);
  if (g_prev.sa_flags & SA_SIGINFO) {
    if (g_prev.sa_sigaction) g_prev.sa_sigaction(sig, info, uc);
  } else if (g_prev.sa_handler != SIG_DFL && g_prev.sa_handler != SIG_IGN) {
    g_prev.sa_handler(sig);
  }
  raise(sig);
}

int segv_bt_install(int fd) {
  if (fd >= 0) g_fd = fd;
  struct sigaction cur;
  if (sigaction(SIGSEGV, NULL, &cur) == 0 && (cur.sa_flags & SA_SIGINFO) && cur.sa_sigaction == on_segv)
    return 0;  /* already in front */
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  return sigaction(SIGSEGV, &sa, &g_prev);
}
