// Build provenance of libgpmpc_mi355x.so (Makefile IDFLAGS): the sha256 of the sources the library
// was compiled from, the git commit it was built at and the build kind.  gpmpc/_lib.py compares the
// hash with the tree it loads the library from, so a stale or A/B-variant library fails loudly.
#ifndef GPMPC_SRC_HASH
#define GPMPC_SRC_HASH "unknown"
#endif
#ifndef GPMPC_GIT_HEAD
#define GPMPC_GIT_HEAD "unknown"
#endif
#ifndef GPMPC_BUILD_KIND
#define GPMPC_BUILD_KIND "unknown"
#endif

extern "C" const char* gpmpc_build_id(void) {
    return "src=" GPMPC_SRC_HASH " git=" GPMPC_GIT_HEAD " kind=" GPMPC_BUILD_KIND;
}
