/* Debug aid (not product code): on SIGSEGV / SIGABRT print the native backtrace (glibc execinfo,
 * addresses as lib+offset) to stderr, then re-raise with the default action.  Runs on an alternate
 * signal stack (a stack overflow leaves none), backtrace() primed at install time (its first call
 * loads libgcc_s).  Loaded with ctypes.CDLL by tools/capture_fork_repro.py; map the offsets with
 * llvm-objdump / nm on the same image's libraries. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static void on_fatal(int sig, siginfo_t *si, void *uc) {
  (void)uc;
  void *buf[128];
  const int n = backtrace(buf, 128);
  static const char hdr[] = "\n=== native backtrace (segv_bt) ===\n";
  if (write(2, hdr, sizeof(hdr) - 1) < 0) return;
  char line[64];
  const unsigned long long a = (unsigned long long)si->si_addr;
  int k = 0;
  line[k++] = 'a'; line[k++] = 'd'; line[k++] = 'd'; line[k++] = 'r'; line[k++] = ' ';
  for (int s = 60; s >= 0; s -= 4) line[k++] = "0123456789abcdef"[(a >> s) & 15];
  line[k++] = '\n';
  if (write(2, line, k) < 0) return;
  backtrace_symbols_fd(buf, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

void segv_bt_install(void) {
  void *prime[4];
  backtrace(prime, 4);
  stack_t ss;
  ss.ss_sp = malloc(1 << 20);
  ss.ss_size = 1 << 20;
  ss.ss_flags = 0;
  sigaltstack(&ss, NULL);
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_fatal;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, NULL);
  sigaction(SIGABRT, &sa, NULL);
  sigaction(SIGBUS, &sa, NULL);
}
