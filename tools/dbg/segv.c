// Debug aid: print a native backtrace on SIGSEGV (load with ctypes.CDLL).
// The handler runs on an alternate signal stack, so a stack overflow (deep
// recursion) is reported too, with the faulting address and the stack bounds.
#define _GNU_SOURCE
#include <execinfo.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
static void handler(int sig, siginfo_t* si, void* uc) {
  (void)uc;
  char msg[160];
  pthread_attr_t at;
  void* sb = 0;
  size_t ss = 0;
  if (pthread_getattr_np(pthread_self(), &at) == 0) {
    pthread_attr_getstack(&at, &sb, &ss);
    pthread_attr_destroy(&at);
  }
  int n = snprintf(msg, sizeof msg, "[segv] signal %d at address %p; thread stack [%p, %p)\n", sig, si->si_addr, sb,
                   (char*)sb + ss);
  write(2, msg, n);
  void* buf[96];
  n = backtrace(buf, 96);
  backtrace_symbols_fd(buf, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
void segv_install(void) {
  static char* alt = 0;
  if (!alt) {
    alt = malloc(1 << 20);
    stack_t st;
    st.ss_sp = alt;
    st.ss_size = 1 << 20;
    st.ss_flags = 0;
    sigaltstack(&st, 0);
  }
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGBUS, &sa, 0);
}
__attribute__((constructor)) static void install_at_load(void) { segv_install(); }
