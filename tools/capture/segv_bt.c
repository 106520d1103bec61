/* segv_bt — diagnostic: on SIGSEGV print the native backtrace (glibc
 * backtrace_symbols_fd) to stderr, then re-raise.  Loaded into a test child
 * with ctypes (tests/capture_child.py, SEGV_BT=path). */
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static void on_segv(int sig) {
  void* frames[64];
  int n = backtrace(frames, 64);
  const char msg[] = "\n[segv_bt] native backtrace:\n";
  if (write(2, msg, sizeof msg - 1) < 0) _exit(139);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void install(void) {
  /* an alternate stack, so a stack overflow is reported too */
  stack_t ss;
  ss.ss_sp = malloc(1 << 20);
  ss.ss_size = 1 << 20;
  ss.ss_flags = 0;
  sigaltstack(&ss, 0);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_segv;
  sa.sa_flags = SA_ONSTACK;
  sigaction(SIGSEGV, &sa, 0);
}
