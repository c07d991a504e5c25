/*
 * bjxa_hip.h -- device-resident extension of libbjxa (symbol version
 * LIBBJXA_HIP_0.1).  New entry points only; nothing in bjxa.h changes.
 *
 * The reference has one hot-path entry per direction, bjxa_decode()
 * (src/libbjxa.c:602-661) and bjxa_encode() (:759-819), both on host
 * buffers, one stream at a time.  These entries take device pointers so a
 * caller that keeps streams in HBM pays no PCIe copy, and accept an
 * explicit entry state -- the same thing the reference expresses through
 * the befL/befR header fields (:417-420) to resume or segment a stream.
 *
 * All pointers named d_* are device pointers on the current HIP device;
 * `stream` is a hipStream_t (NULL = default stream).  Calls are
 * asynchronous; results are valid once the stream has been synchronized.
 * Return: 0, or -1 with errno (EINVAL bad argument/alignment, ENODEV no
 * GPU, EIO launch failure).
 */
#ifndef BJXA_HIP_H_INCLUDED
#define BJXA_HIP_H_INCLUDED

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* one stream to decode */
typedef struct {
	const void	*d_src;		/* XA blocks (no header), 4-B aligned */
	void		*d_dst;		/* PCM out, 16-B aligned */
	uint64_t	frames;		/* frames to emit: (eblocks-1)*32 <
					 * frames <= eblocks*32 */
	uint32_t	eblocks;	/* effective blocks */
	uint8_t		bits;		/* 4, 6 or 8 */
	uint8_t		channels;	/* 1 or 2 */
	int16_t		state[4];	/* entry state: L prev[0], L prev[1],
					 * R prev[0], R prev[1] */
} bjxa_hip_stream_t;

/* tuning and profiling hooks (zero/NULL = automatic/off) */
typedef struct {
	uint32_t	chunk;		/* eblocks per lane */
	int32_t		warmup;		/* speculative warm-up eblocks, -1 = auto */
	void		*ev_spec[2];	/* hipEvent_t pair recorded on `stream`
					 * around the speculative-decode kernel */
	uint32_t	variant;	/* bits 8-11: pacing of the speculative
					 * kernel's waves (0 = automatic, 15 =
					 * off, n = a barrier every n groups);
					 * batches: bit 16 forces, bit 17
					 * forbids the longer chunks planned
					 * for packed PCM images (automatic:
					 * by layout); test knobs of the
					 * verify pass: bit 18 makes every
					 * wave leave its first boundary to
					 * the sequential tail, bit 19 stops
					 * waves waiting for the exit record
					 * of the wave before them; bit 20:
					 * the caller keeps two decodes in
					 * flight, plan for one decode-kernel
					 * workgroup per CU (chunks twice as
					 * long); other bits reserved (0).
					 * Pass the same tuning to
					 * bjxa_hip_decode_workspace. */
} bjxa_hip_tuning_t;

/*
 * Status written by a decode (8 x uint32, device memory):
 *  [0] first failing channel block (eblock*channels + channel) whose gain
 *      nibble is >= 5, 0xffffffff if none (the reference's EPROTO, :550)
 *  [1] exit state L (prev[0] | prev[1] << 16)
 *  [2] exit state R
 *  [3] chunks repaired inside the decode kernel, [4] by the sequential
 *      tail (cascades, and boundaries the decode kernel left to it),
 *  [5] chunks, [6] chunk length and [7] warm-up length used (eblocks)
 */
#define BJXA_HIP_STATUS_WORDS 8

/* workspace bytes for one stream of `eblocks`, non-decreasing in `eblocks`
 * under the automatic plan (tune == NULL or tune->chunk == 0), so the same
 * workspace serves every shorter stream too; call bjxa_hip_workspace_init
 * once before first use; a completed decode leaves it reusable.  A decode
 * whose launch fails re-initialises it itself; after a device fault (an
 * error from the stream) initialise it again before reusing it */
size_t bjxa_hip_decode_workspace(uint32_t eblocks, unsigned channels,
    const bjxa_hip_tuning_t *tune);
int bjxa_hip_workspace_init(void *d_ws, size_t ws_len, void *stream);

/* decode one stream (two kernels on `stream`, no host sync) */
int bjxa_hip_decode_async(const bjxa_hip_stream_t *s, void *d_ws,
    size_t ws_len, uint32_t *d_status, const bjxa_hip_tuning_t *tune,
    void *stream);

/*
 * Batched decode: n independent streams (any mix of bits and channels) in
 * one launch per kernel -- SURVEY.md §8(d) C4/C5.  bjxa_hip_batch_new
 * validates the streams, plans chunks, allocates the batch's device
 * workspace and uploads its tables (the descriptors, including the device
 * buffers they name, are captured: re-create the batch for other buffers).
 * Each decode writes n status records of BJXA_HIP_STATUS_WORDS words
 * (stream i at d_status + 8*i) with the meaning above; tune (optional)
 * supplies only the profiling events.  Tuning at creation: chunk = channel
 * blocks per lane (0 = automatic), warmup.
 */
typedef struct bjxa_hip_batch bjxa_hip_batch_t;
bjxa_hip_batch_t *bjxa_hip_batch_new(const bjxa_hip_stream_t *s, uint32_t n,
    const bjxa_hip_tuning_t *tune, void *stream);
int bjxa_hip_batch_decode_async(bjxa_hip_batch_t *b, uint32_t *d_status,
    const bjxa_hip_tuning_t *tune, void *stream);
void bjxa_hip_batch_free(bjxa_hip_batch_t *b);

/*
 * Decode n complete XA files (32-byte header + blocks) held in host memory
 * into n complete WAV files (44-byte RIFF header + PCM) with one batched
 * GPU pass.  wav[i] needs 44 + data_len_pcm bytes.  status[i]: 0, EPROTO
 * (bad header, or a block profile with gain >= 5: the WAV then holds the
 * PCM before it), ENOBUFS (input shorter than announced, output too small)
 * or EFAULT.  Returns the number of files decoded completely, or -1 with
 * errno if the batch itself fails.
 */
int bjxa_hip_decode_files(const void *const *xa, const size_t *xa_len,
    void *const *wav, const size_t *wav_len, int *status, uint32_t n);

/* encode `frames` frames of 16-bit PCM into ceil(frames/32) XA eblocks
 * (profile 0, last block zero-padded), d_pcm 16-B aligned, d_xa 4-B */
int bjxa_hip_encode_async(const void *d_pcm, uint64_t frames, unsigned bits,
    unsigned channels, void *d_xa, void *stream);

/*
 * Validate n XA headers held in device memory (32 bytes each, header i at
 * d_src + i * stride; any alignment) with the checks, order and uint32
 * arithmetic of bjxa_parse_header (src/libbjxa.c:395-453), one thread per
 * header, and write one record each (LIBBJXA_HIP_0.2).  A stereo header
 * whose payload is an odd number of channel blocks passes the reference's
 * checks and then trips its format assertion (:597); here it is EPROTO.
 * For batches of files already in HBM (10^5 and more).
 */
typedef struct {
	uint32_t	data_len;	/* XA block bytes (nDataLen) */
	uint32_t	samples;	/* frames (nSamples) */
	uint32_t	blocks;		/* effective blocks */
	uint32_t	data_len_pcm;	/* samples * channels * 2 */
	uint16_t	rate;
	uint8_t		bits;
	uint8_t		channels;
	int16_t		state[4];	/* befL[0..1], befR[0..1] */
	int32_t		status;		/* 0 or EPROTO; the rest is 0 on EPROTO */
} bjxa_hip_header_t;		/* 32 bytes */

int bjxa_hip_parse_headers_async(const void *d_src, size_t stride, uint32_t n,
    bjxa_hip_header_t *d_out, void *stream);

/*
 * Routing of the host API (LIBBJXA_HIP_0.3).  bjxa_decode()/bjxa_encode()
 * run a call of at least `eblocks` effective blocks on the GPU and a
 * smaller one on the calling thread's CPU core; without a GPU every call
 * runs on the CPU.  0 sends every call to the GPU, INT64_MAX none.
 * eblocks < 0 only queries.  Returns the previous threshold, or -1/EINVAL
 * for an unknown direction.  Process-wide and thread-safe; the defaults
 * (measured crossover points, DESIGN.md §1: 1,024 eblocks for decode,
 * 4,096 for encode) can be overridden with the environment variables
 * BJXA_OFFLOAD_DECODE / BJXA_OFFLOAD_ENCODE.
 */
#define BJXA_HIP_OFFLOAD_DECODE	0
#define BJXA_HIP_OFFLOAD_ENCODE	1
int64_t bjxa_hip_offload_threshold(int direction, int64_t eblocks);

/* library/kernels build identifier, e.g. "bjxa-mi355x gfx950 ..." */
const char *bjxa_hip_version(void);

#ifdef __cplusplus
}
#endif

#endif /* BJXA_HIP_H_INCLUDED */
