/* Debug aid (not product code): on SIGSEGV / SIGABRT print the native backtrace (glibc execinfo,
 * addresses as lib+offset) to stderr, then re-raise with the default action.  Loaded with
 * ctypes.CDLL by tools/capture_fork_repro.py; map the offsets with llvm-objdump / nm on the
 * same image's libraries. */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_fatal(int sig) {
  void *buf[96];
  const int n = backtrace(buf, 96);
  static const char hdr[] = "\n=== native backtrace (segv_bt) ===\n";
  if (write(2, hdr, sizeof(hdr) - 1) < 0) return;
  backtrace_symbols_fd(buf, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

/* called by the loader after torch / the HIP runtime have installed their own handlers */
void segv_bt_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_handler = on_fatal;
  sigaction(SIGSEGV, &sa, NULL);
  sigaction(SIGABRT, &sa, NULL);
}
