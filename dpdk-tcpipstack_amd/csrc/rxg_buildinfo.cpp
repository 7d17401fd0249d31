// rxg_build_info (include/rxg.h): which sources this library was built from.
// build/buildid.h is written by the Makefile: RXG_SRC_HASH is the first 16 hex digits of
// sha256 over every product source (csrc/*.h, *.hip, *.cpp in sorted order, then
// include/rxg.h), which rxg.source_hash() recomputes from a tree to tell a stale library
// from a current one; RXG_GIT_REV is the checkout's revision (+dirty when csrc/ or include/
// differ from it).
#include "rxg.h"
#include "buildid.h"

extern "C" const char *rxg_build_info(void)
{
    return "rxg src=" RXG_SRC_HASH " rev=" RXG_GIT_REV " built=" __DATE__ " " __TIME__ " gfx950";
}
