/*
 * action_1 -- the one-argument callback record used by every byte stream.
 *
 * Drop-in boundary type.  The layout ({void *obj; act_1 act;}, passed by
 * value) must stay identical to the reference's, see
 * /root/reference/include/action_1.h:10-20, because bytestream_1 vtables
 * (include/bytestream_1.h) carry it across the C ABI.
 */
#ifndef ASYNC_AMD_ACTION_1_H
#define ASYNC_AMD_ACTION_1_H

#ifdef __cplusplus
extern "C" {
#endif

typedef void (*act_1)(void *obj);

typedef struct {
    void *obj;
    act_1 act;
} action_1;

/* Invoke the callback.  (ref: include/action_1.h:15-18) */
static inline void action_1_perf(action_1 action)
{
    action.act(action.obj);
}

/* A callback that does nothing; the "no callback registered" value.
 * (ref: src/action_1.c:12) */
extern action_1 NULL_ACTION_1;

#ifdef __cplusplus
}
#endif

#endif /* ASYNC_AMD_ACTION_1_H */
