/*
 * xa_gpu.h -- internal interface between the host C library (libbjxa.c)
 * and the HIP translation units.  Local symbols; not part of the ABI.
 */
#ifndef BJXA_XA_GPU_H
#define BJXA_XA_GPU_H

#include <stddef.h>
#include <stdint.h>

#include "bjxa_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

struct bjxa__gpu;

/* NULL + errno (ENODEV without a GPU, ENOMEM) on failure */
/* a HIP device is visible (checked once) */
int bjxa__gpu_present(void);

struct bjxa__gpu *bjxa__gpu_new(void);
void bjxa__gpu_free(struct bjxa__gpu *g);

/*
 * Decode `eblocks` effective blocks from host `src`, starting in `state`
 * (L p0, L p1, R p0, R p1); copy the first `dst_bytes` PCM bytes to host
 * `dst`.  *err_cb is the first failing channel block (eblock*ch + channel)
 * or 0xffffffff; on failure only the eblocks before it are copied and
 * `state` is the state at that point.  Returns 0 or -1/errno.
 */
int bjxa__gpu_decode(struct bjxa__gpu *g, const void *src, uint32_t eblocks,
    unsigned bits, unsigned ch, int16_t state[4], void *dst,
    uint64_t dst_bytes, uint32_t *err_cb);

/* one stream of a many-file decode (bjxa_hip_decode_files) */
struct bjxa__job {
	const void	*src;		/* host XA blocks */
	void		*dst;		/* host PCM destination */
	uint64_t	dst_bytes;	/* PCM bytes wanted (the last block may be cut) */
	uint32_t	eblocks;
	uint8_t		bits, ch;
	int16_t		state[4];
	uint32_t	err_cb;		/* out: as bjxa__gpu_decode */
};

/*
 * Decode n independent streams from host memory in one batched pass
 * (bjxa_hip_batch_*); each job's PCM lands in its dst, up to the first
 * failing eblock.  Returns 0 or -1/errno (ENODEV, ENOMEM, EIO).
 */
int bjxa__gpu_decode_many(struct bjxa__job *jobs, uint32_t n);

/* bjxa_hip_batch_new in a device workspace the caller keeps across
 * batches (grown in place; not freed by bjxa_hip_batch_free) */
bjxa_hip_batch_t *bjxa__batch_new(const bjxa_hip_stream_t *s, uint32_t n,
    const bjxa_hip_tuning_t *tune, void *stream, void **ws_cache,
    size_t *ws_cap);

/* encode `frames` frames from host `src` into ceil(frames/32) eblocks */
int bjxa__gpu_encode(struct bjxa__gpu *g, const void *src, uint64_t frames,
    unsigned bits, unsigned ch, void *dst);

/*
 * CPU core (xa_cpu.c): the same contracts as bjxa__gpu_decode and
 * bjxa__gpu_encode, on the calling thread; they cannot fail.
 */
int bjxa__cpu_decode(const void *src, uint32_t eblocks, unsigned bits,
    unsigned ch, int16_t state[4], void *dst, uint64_t dst_bytes,
    uint32_t *err_cb);
int bjxa__cpu_encode(const void *src, uint64_t frames, unsigned bits,
    unsigned ch, void *dst);

#ifdef __cplusplus
}
#endif

#endif
