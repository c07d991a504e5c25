/*
 * xa_gpu_none.c -- the GPU side of xa_gpu.h for a host-only build (make
 * sanitize): no device is ever present, so libbjxa.c routes every call to
 * the CPU core (xa_cpu.c).  Lets the host C run under ASan/UBSan, which the
 * GPU code objects cannot (reference configure.ac:41-43,66-75
 * builds its own sanitizer variant the same way).  Not part of the shipped
 * library.
 */
#include <errno.h>
#include <stddef.h>

#include "xa_gpu.h"

int
bjxa__gpu_present(void)
{
	return 0;
}

struct bjxa__gpu *
bjxa__gpu_new(void)
{
	errno = ENODEV;
	return NULL;
}

void
bjxa__gpu_free(struct bjxa__gpu *g)
{
	(void)g;
}

int
bjxa__gpu_decode(struct bjxa__gpu *g, const void *src, uint32_t eblocks,
    unsigned bits, unsigned ch, int16_t state[4], void *dst,
    uint64_t dst_bytes, uint32_t *err_cb)
{
	(void)g, (void)src, (void)eblocks, (void)bits, (void)ch, (void)state;
	(void)dst, (void)dst_bytes, (void)err_cb;
	errno = ENODEV;
	return -1;
}

int
bjxa__gpu_decode_many(struct bjxa__job *jobs, uint32_t n)
{
	(void)jobs, (void)n;
	errno = ENODEV;
	return -1;
}

int
bjxa__gpu_encode(struct bjxa__gpu *g, const void *src, uint64_t frames,
    unsigned bits, unsigned ch, void *dst)
{
	(void)g, (void)src, (void)frames, (void)bits, (void)ch, (void)dst;
	errno = ENODEV;
	return -1;
}
