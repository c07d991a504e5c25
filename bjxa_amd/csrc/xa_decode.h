/*
 * xa_decode.h -- kernel argument block and workspace layout (internal).
 */
#ifndef BJXA_XA_DECODE_H
#define BJXA_XA_DECODE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

/* xa_dec_args::flags, test knobs of the verify pass (tuning variant bits
 * 18 and 19, include/bjxa_hip.h) */
#define XA_F_NORECORD	1u	/* no exit records: every wave's first boundary
				 * goes to the sequential tail */
#define XA_SPIN_TICKS	20000u	/* default xa_dec_args::spin (200 us); tuning
				 * variant bit 19 sets 0 */

/* workspace control words (reset by the tail kernel after every call) */
#define XA_CTL_ERR	0	/* min channel-block index with gain >= 5 */
#define XA_CTL_NQ	1	/* entries appended to the re-check queue */
#define XA_CTL_FIXED	2	/* chunks repaired */
#define XA_CTL_OVF	3	/* the queue overflowed (a workspace left
				 * inconsistent by a failed launch): the tail
				 * re-checks every chunk boundary */
#define XA_CTL_WORDS	64	/* 256 B */

/* status words written by the tail kernel */
#define XA_ST_ERR	0
#define XA_ST_STATE_L	1
#define XA_ST_STATE_R	2
#define XA_ST_FIXED	3
#define XA_ST_TAIL	4
#define XA_ST_CHUNKS	5
#define XA_ST_C		6
#define XA_ST_W		7
#define XA_ST_WORDS	8

/*
 * Chunk and warm-up lengths are whole multiples of this many eblocks (8
 * channel blocks): K1 moves a lane's input two groups of 4 channel blocks
 * at a time.
 */
#define XA_CHUNK_Q(ch)	(8u / (ch))

struct xa_dec_args {
	const uint8_t *src;	/* XA blocks, eblock b at src + b*ch*(bits*4+1) */
	uint8_t *dst;		/* PCM, eblock b at dst + b*64*ch */
	uint64_t pcm_bytes;	/* PCM bytes to emit (last block may be cut) */
	uint32_t eblocks;
	uint32_t nchunks;
	uint32_t C, W;		/* chunk and warm-up lengths in eblocks
				 * (multiples of XA_CHUNK_Q(ch)); chunk q
				 * starts at eblock q*C */
	uint32_t init[2];	/* caller state per channel, p0 | p1 << 16 */
	const uint32_t *init_dev; /* if not NULL: the entry state is read from
				 * these status words (XA_ST_STATE_L/R) of
				 * the decode before, in stream order, instead
				 * of init (xa_gpu.hip duplex_decode's slabs) */
	uint32_t pace;		/* K1 waves of a workgroup wait for each other
				 * every `pace` groups (0 = never) */
	uint2 *g, *e;		/* per-chunk entry / exit state, as repaired */
	uint32_t *queue;	/* chunks for the tail to re-check in order
				 * (entry = qbase + chunk; batches: the batch's
				 * queue, global chunk indices) */
	uint32_t *nq;		/* its length (ctl[XA_CTL_NQ] of the launch) */
	uint32_t qcap;		/* its capacity in entries */
	uint32_t qbase;		/* the stream's first global chunk */
	uint32_t *ovf;		/* ctl[XA_CTL_OVF] of the launch */
	uint4 *exits;		/* per wave of the stream: the exit state its
				 * last chunk left, tagged (xa_decode.hip) */
	uint32_t tag;		/* this launch's record tag, never 0 */
	uint32_t spin;		/* 100-MHz ticks a wave waits for the record
				 * of the wave before it */
	uint32_t flags;		/* XA_F_* */
	uint32_t *ctl;		/* XA_CTL_WORDS */
	uint32_t *status;	/* XA_ST_WORDS */
};

/*
 * The decode kernel (decode, verify and repair every chunk boundary it can
 * see, including the one with the previous wave) and the tail kernel
 * (cascades and what the first could not settle, in chunk order; status) on
 * `st`; ev0/ev1 (optional) around the first.
 */
hipError_t xa_decode_launch(const xa_dec_args &a, unsigned bits, unsigned ch,
    hipStream_t st, hipEvent_t ev0, hipEvent_t ev1);

/*
 * Batched decode: many independent streams, mixed formats, one launch per
 * kernel.  Every stream's chunks occupy whole waves of a global chunk index
 * space (stream i owns global chunks [cbase, cbase + 64 * waves_i)), so
 * wave w belongs to stream wstream[w] and takes its chunks 64w - cbase ..
 * +63.
 */
struct xa_batch_stream {		/* 64 B, device table entry */
	const uint8_t *src;
	uint8_t *dst;
	uint64_t pcm_bytes;
	uint32_t eblocks, nchunks;
	uint32_t cbase;			/* first global chunk, % 64 == 0 */
	uint32_t C;			/* chunk length, eblocks */
	uint32_t init[2];
	uint32_t fmt;			/* bits | channels << 8 */
	uint32_t pad[3];
};

/* per-stream control words (xa_batch_args::sctl); ERR and FIXED sit where
 * xa_dec_args::ctl has them, so a stream's sctl serves as its ctl */
#define XA_SCTL_ERR	0
#define XA_SCTL_TAIL	1
#define XA_SCTL_FIXED	2
#define XA_SCTL_WORDS	4

struct xa_batch_args {
	const xa_batch_stream *streams;
	const uint32_t *wstream;	/* stream of each wave */
	uint32_t nstreams, nwaves;	/* global chunks = 64 * nwaves */
	uint32_t W;
	uint32_t pace;			/* as xa_dec_args::pace */
	uint2 *g, *e;			/* per global chunk */
	uint32_t *queue;		/* 2 * 64 * nwaves */
	uint4 *exits;			/* per global wave (xa_dec_args::exits) */
	uint32_t tag, spin, flags;	/* as xa_dec_args */
	uint32_t *ctl;			/* XA_CTL_WORDS (NQ, OVF) */
	uint32_t *sctl;			/* XA_SCTL_WORDS per stream */
	uint32_t *status;		/* XA_ST_WORDS per stream */
};

hipError_t xa_decode_batch_launch(const xa_batch_args &b, hipStream_t st,
    hipEvent_t ev0, hipEvent_t ev1);

/*
 * Low-latency path for small host-API calls (xa_small.hip): input, PCM and
 * status in one pinned, device-mapped host buffer per codec.
 */
#define XA_SMALL_MAX	32	/* eblocks per call */
#define XA_SMALL_IN	4096	/* input area (XA or PCM) */
#define XA_SMALL_STATUS	4096	/* status words, offset within the output area */
#define XA_SMALL_BYTES	(XA_SMALL_IN + XA_SMALL_STATUS + 64)

hipError_t xa_small_decode_launch(const uint8_t *in_h, uint8_t *out_h,
    uint32_t n, unsigned bits, unsigned ch, const uint32_t init[2],
    hipStream_t st);
hipError_t xa_small_encode_launch(const uint8_t *in_h, uint8_t *out_h,
    uint64_t frames, unsigned bits, unsigned ch, hipStream_t st);

struct xa_enc_args {
	const uint8_t *src;	/* PCM frames, 16-bit, channels interleaved */
	uint8_t *dst;		/* XA blocks */
	uint64_t frames;	/* valid frames; the last block is zero-padded */
	uint32_t eblocks;	/* ceil(frames / 32) */
};

hipError_t xa_encode_launch(const xa_enc_args &a, unsigned bits, unsigned ch,
    hipStream_t st);

#endif
