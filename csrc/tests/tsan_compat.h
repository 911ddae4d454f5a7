// Force-included into the ThreadSanitizer build of the host tests only.
// libstdc++ (GCC 11) waits on condition variables with pthread_cond_clockwait,
// which this libtsan does not intercept: TSan then believes a waiting thread
// still holds the mutex and reports bogus "double lock" / races on every
// condition-variable hand-off.  Falling back to pthread_cond_timedwait keeps
// the analysis exact for the code under test.
#pragma once
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
