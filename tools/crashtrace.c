/* Debug aid: on SIGSEGV/SIGABRT print the native backtrace (dladdr symbols) to stderr, then die
 * with the default action. Built by tools/crashtrace.sh, loaded by probes via ctypes. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fault(int sig, siginfo_t* si, void* uc) {
  (void)uc;
  void* frames[64];
  char msg[96];
  int n = backtrace(frames, 64);
  int len = 0;
  const char* hdr = "\n=== crashtrace: signal ";
  write(2, hdr, strlen(hdr));
  len = 0;
  msg[len++] = '0' + (sig / 10) % 10;
  msg[len++] = '0' + sig % 10;
  msg[len++] = '\n';
  write(2, msg, len);
  (void)si;
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void crashtrace_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_fault;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGABRT, &sa, 0);
  sigaction(SIGBUS, &sa, 0);
}
