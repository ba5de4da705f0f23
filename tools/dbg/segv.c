// Debug aid: print a native backtrace on SIGSEGV (load with ctypes.CDLL).
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>
static void handler(int sig) {
  void* buf[64];
  int n = backtrace(buf, 64);
  backtrace_symbols_fd(buf, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
void segv_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = handler;
  sigaction(SIGSEGV, &sa, 0);
}
__attribute__((constructor)) static void install_at_load(void) { segv_install(); }
