// lsg_ab.h -- the A/B and test switches.  The shipped library (liblodestar_bls.so) reads no
// environment variable that changes arithmetic or verdict flow: every switch below is a
// compile-time constant there.  The A/B build (liblodestar_bls_ab.so, compiled with -DLSG_AB
// by lodestar_amd/build.py: tests that compare two forms of a stage, bench A/B runs) reads
// them from the environment per call, so one process can compare both forms.
#pragma once
#include <stdlib.h>
#include <string.h>

#ifdef LSG_AB
// integer switch `name`, `dflt` when unset
static inline long lsg_ab_long(const char* name, long dflt) {
  const char* e = getenv(name);
  return e ? atol(e) : dflt;
}
static inline bool lsg_ab_str_is(const char* name, const char* v) {
  const char* e = getenv(name);
  return e && strcmp(e, v) == 0;
}
#else
#define lsg_ab_long(name, dflt) ((long)(dflt))
#define lsg_ab_str_is(name, v) false
#endif
