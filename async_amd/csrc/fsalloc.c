/*
 * fsalloc.c -- the object allocator of the standalone library
 * (include/fsalloc.h).  Not part of libasync_b64_core.so: in a reference
 * build fsdyn supplies these calls.
 *
 * Every allocation and free goes through one replaceable realloc-like
 * function, which is what lets a test runner count live objects the way
 * the reference's does (test/asynctest.c:111-147).
 */
#include <stdlib.h>
#include <string.h>

#include "fsalloc.h"

static void *default_realloc(void *ptr, size_t size)
{
    if (size == 0) {
        free(ptr);
        return NULL;
    }
    return realloc(ptr, size);
}

static fs_realloc_t reallocator = default_realloc;
static void (*realloc_counter)(int);

void *fsalloc(size_t size)
{
    void *p = reallocator(NULL, size ? size : 1);
    if (!p)
        abort(); /* the reference's allocation failure is fatal */
    return p;
}

void *fscalloc(size_t nmemb, size_t size)
{
    if (size && nmemb > (size_t) -1 / size)
        abort();
    size_t total = nmemb * size;
    void *p = fsalloc(total);
    memset(p, 0, total);
    return p;
}

void fsfree(void *ptr)
{
    if (ptr)
        (void) reallocator(ptr, 0);
}

fs_realloc_t fs_get_reallocator(void)
{
    return reallocator;
}

void fs_set_reallocator(fs_realloc_t r)
{
    reallocator = r ? r : default_realloc;
}

void fs_set_reallocator_counter(void (*counter)(int))
{
    realloc_counter = counter;
}
