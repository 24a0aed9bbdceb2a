/*
 * fsalloc.h -- the object allocator of the reference's ecosystem, as far as
 * this library and the reference's tests use it.
 *
 * The reference allocates every object with fsalloc() (e.g.
 * src/nicestream.c:119) and its loop frees wounded objects with fsfree()
 * (src/async.c:127-130, via async_wound() :386-392).  Both come from the
 * external fsdyn library (<fsdyn/fsalloc.h>, not vendored, SURVEY.md §2 row
 * 15).  The reference's test runner swaps the allocator for a counting one
 * (test/asynctest.c:111-147, 276-278) and fails a test that leaves objects
 * outstanding.
 *
 * So an object handed to async_wound() must come from fsalloc():
 *  - libasync_b64_core.so (the drop-in for a reference build) leaves fsalloc
 *    and fsfree undefined; the reference's own fsdyn provides them, and the
 *    stages' objects are counted and freed by the reference's allocator;
 *  - libasync_b64.so (standalone, with its own loop) defines the calls
 *    below (async_amd/csrc/fsalloc.c), and its loop's async_wound() frees
 *    through fsfree(), so the same counting allocator can be wired in the
 *    same way (tests/test_stage_fake.py::test_reference_topology_leak_check).
 *
 * Only the names the reference itself uses are declared here.  Allocation
 * failure aborts, as in the reference ("Errors").
 */
#ifndef ASYNC_AMD_FSALLOC_H
#define ASYNC_AMD_FSALLOC_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* realloc(3)-like: (NULL, n) allocates, (p, 0) frees and returns NULL. */
typedef void *(*fs_realloc_t)(void *ptr, size_t size);

void *fsalloc(size_t size);
void *fscalloc(size_t nmemb, size_t size);
void fsfree(void *ptr);

fs_realloc_t fs_get_reallocator(void);
void fs_set_reallocator(fs_realloc_t reallocator);
/* Called with +n / -n for objects the library accounts for outside the
 * reallocator (this library has none; kept for the test runner's wiring,
 * test/asynctest.c:132-135, 278). */
void fs_set_reallocator_counter(void (*counter)(int count));

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_FSALLOC_H */
