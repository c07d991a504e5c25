/*
 * pattern_probe.hip -- read rate of the decode's input access pattern,
 * isolated from the decode: every lane owns one "chunk" (a contiguous run of
 * CB bytes) and walks it in steps of SEG bytes; a wave stages one step of its
 * 64 lanes into LDS by 16-B LDS-DMA with the 64 segments concatenated (the
 * K1 scheme), then every lane reads its segment back.  Variants:
 *   SEG   bytes per lane per step (144 = K1's 8-bit group slot)
 *   DEPTH steps in flight per wave (1: wait, consume, issue the next)
 * plus a contiguous control (chunks interleaved so each DMA instruction reads
 * 1 KiB of contiguous source).  Total bytes and waves match C3 (330 MB,
 * 125,000 lanes).  Prints JSON lines.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -o pattern_probe tools/pattern_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ void
dma16(const void *g, uint8_t *l)
{
	__builtin_amdgcn_global_load_lds(g, LDS_PTR(l), 16, 0, 0);
}

template <int SEG, int DEPTH, bool CONTIG>
__global__ __launch_bounds__(256) void
k_pattern(const uint8_t *src, uint32_t *sink, uint32_t CB, uint32_t steps)
{
	constexpr int NP = SEG / 16;
	__shared__ __attribute__((aligned(16))) uint8_t lds[4 * DEPTH * 64 * SEG];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	uint8_t *reg = lds + wv * DEPTH * 64 * SEG;
	const uint64_t w = blockIdx.x * 4u + wv;
	/* source byte of piece i of step s: strided chunks (lane t's segment at
	 * chunk t, offset s*SEG) or contiguous (the wave's step s is one run
	 * of 64*SEG bytes) */
	uint32_t voff[NP];
#pragma unroll
	for (int i = 0; i < NP; i++) {
		const int k = i * 64 + lane;
		voff[i] = CONTIG ? (uint32_t)k * 16u :
		    (uint32_t)(k / NP) * CB + (uint32_t)(k % NP) * 16u;
	}
	const uint8_t *wbase = src + w * 64ull * CB;
	auto issue = [&](uint32_t s) {
		const uint8_t *b = wbase + (CONTIG ? (uint64_t)s * 64 * SEG :
		    (uint64_t)s * SEG);
		uint8_t *l = reg + (s % DEPTH) * 64 * SEG;
#pragma unroll
		for (int i = 0; i < NP; i++)
			dma16(b + voff[i], l + i * 64 * 16);
	};
	uint32_t acc = 0;
#pragma unroll
	for (int d = 0; d < DEPTH - 1; d++)
		issue(d);
	for (uint32_t s = 0; s < steps; s++) {
		if (s + DEPTH - 1 < steps)
			issue(s + DEPTH - 1);
		if (DEPTH == 1)
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		else if (DEPTH == 2)
			asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NP) : "memory");
		else
			asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NP) : "memory");
		if (s + DEPTH - 1 >= steps)
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		const uint32_t *m = (const uint32_t *)(reg + (s % DEPTH) * 64 * SEG +
		    lane * SEG);
#pragma unroll
		for (int i = 0; i < SEG / 4; i++)
			acc += m[i];
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		__builtin_amdgcn_wave_barrier();
	}
	if (acc == 0x9e3779b9u)
		*sink = acc;
}

template <int SEG, int DEPTH, bool CONTIG>
static void
run(const uint8_t *src, uint32_t *sink)
{
	/* 125,000 lanes (1,954 waves, 489 workgroups) as K1 on C3; chunk =
	 * 40 eblocks x 66 B rounded to whole steps */
	const uint32_t lanes = 125056, CB0 = 2640;
	const uint32_t steps = CB0 / SEG, CB = steps * SEG;
	const unsigned grid = lanes / 256;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int i = 0; i < 2; i++)
		hipLaunchKernelGGL((k_pattern<SEG, DEPTH, CONTIG>), dim3(grid), dim3(256), 0, 0, src, sink, CB, steps);
	hipEventRecord(a, 0);
	for (int i = 0; i < 20; i++)
		hipLaunchKernelGGL((k_pattern<SEG, DEPTH, CONTIG>), dim3(grid), dim3(256), 0, 0, src, sink, CB, steps);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	ms /= 20;
	const double bytes = (double)lanes * CB;
	printf("{\"seg\": %d, \"depth\": %d, \"contig\": %d, \"ms\": %.4f, \"TBs\": %.3f}\n",
	    SEG, DEPTH, CONTIG ? 1 : 0, ms, bytes / ms / 1e9);
	hipEventDestroy(a);
	hipEventDestroy(b);
}


/*
 * K1 skeleton: the decode kernel's memory structure with a trivial "decode"
 * (out dword i = in dword i % 33 ^ i): per step a lane consumes one 144-B
 * input slot (132 B used) and emits 256 B (two 128-B lines).  Input: LDS-DMA
 * into two alternating buffers (the next step's DMA issued before the work,
 * counted vmcnt(16) wait).  Output: STAGE = lines staged in the consumed
 * buffer and stored 8 whole lines per instruction (K1), or direct 16-B
 * stores from VGPRs.  SIN/SOUT: lane-chunk strided (K1) or wave-contiguous.
 */
template <bool SIN, bool SOUT, bool STAGE, int PF = 0>
__global__ __launch_bounds__(256) void
k_skel(const uint8_t *src, uint8_t *dst, uint32_t steps)
{
	constexpr int SEG = 144, NP = 9, LINE = 144, RS = 64 * SEG;
	__shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * RS];
	__shared__ __attribute__((aligned(16))) uint8_t pfs[4 * 256];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	uint8_t *reg = lds + wv * 2 * RS;
	const uint64_t w = blockIdx.x * 4u + wv;
	const uint32_t CBI = steps * 132u, CBO = steps * 256u;
	uint32_t voff[NP];
#pragma unroll
	for (int i = 0; i < NP; i++) {
		const int k = i * 64 + lane;
		voff[i] = SIN ? (uint32_t)(k / NP) * CBI + (uint32_t)(k % NP) * 16u :
		    (uint32_t)k * 16u;
	}
	const uint8_t *wbi = src + w * 64ull * CBI;
	uint8_t *wbo = dst + w * 64ull * CBO;
	auto issue = [&](uint32_t s, uint8_t *l) {
		const uint8_t *b = wbi + (SIN ? (uint64_t)s * 132u : (uint64_t)s * 64u * SEG);
#pragma unroll
		for (int i = 0; i < NP; i++)
			dma16(b + voff[i], l + i * 64 * 16);
	};
	issue(0, reg);
	int cur = 0;
	for (uint32_t s = 0; s < steps; s++) {
		uint8_t *cb = reg + (cur ? RS : 0), *ob = reg + (cur ? 0 : RS);
		if (s == 0)
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		else if (PF && ((s - 1) % 4 == 0))
			asm volatile("s_waitcnt vmcnt(21)" ::: "memory");
		else
			asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
		uint32_t win[33];
		const uint32_t *m = (const uint32_t *)(cb + lane * SEG);
#pragma unroll
		for (int i = 0; i < 33; i++)
			win[i] = m[i];
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		if (s + 1 < steps)
			issue(s + 1, ob);
		if (PF && s % 4 == 0) {
			/* pull this lane's input lines of steps s+PF .. s+PF+3 into
			 * the caches in one burst (one dword per 128-B line) */
			const uint8_t *b = src + (w * 64ull + lane) * CBI +
			    (uint64_t)(s + PF) * 132u;
			const uint8_t *lim = src + (w * 64ull + lane + 1) * CBI - 4;
#pragma unroll
			for (int k = 0; k < 5; k++) {
				const uint8_t *a = b + k * 128;
				__builtin_amdgcn_global_load_lds(a < lim ? a : lim,
				    LDS_PTR(pfs + wv * 256), 4, 0, 0);
			}
		}
		asm volatile("" ::: "memory");
#pragma unroll
		for (int h = 0; h < 2; h++) {
			u32x4 v[8];
#pragma unroll
			for (int q = 0; q < 8; q++)
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const int i = h * 32 + q * 4 + j;
					v[q][j] = win[i % 33] ^ (uint32_t)i;
				}
			/* this lane's 128-B line h of step s */
			if (!STAGE) {
				uint8_t *o = SOUT ? wbo + (uint64_t)lane * CBO + s * 256u + h * 128u :
				    wbo + ((uint64_t)(s * 2 + h) * 64u + lane) * 128u;
#pragma unroll
				for (int q = 0; q < 8; q++)
					__builtin_nontemporal_store(v[q], (u32x4 *)(o + q * 16));
				continue;
			}
			uint8_t *line = cb + lane * LINE;
#pragma unroll
			for (int q = 0; q < 8; q++)
				*(u32x4 *)(line + q * 16) = v[q];
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			/* instruction i: lanes 8k..8k+7 store line 8i+k's pieces */
#pragma unroll
			for (int i = 0; i < 8; i++) {
				const int ln = i * 8 + lane / 8, pc = lane % 8;
				const u32x4 x = *(const u32x4 *)(cb + ln * LINE + pc * 16);
				uint8_t *o = SOUT ? wbo + (uint64_t)ln * CBO + s * 256u + h * 128u + pc * 16u :
				    wbo + ((uint64_t)(s * 2 + h) * 64u + ln) * 128u + pc * 16u;
				__builtin_nontemporal_store(x, (u32x4 *)o);
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		cur ^= 1;
	}
}

template <bool SIN, bool SOUT, bool STAGE, int PF = 0>
static void
run_skel(const uint8_t *src, uint8_t *dst)
{
	const uint32_t lanes = 125056, steps = 20;
	const unsigned grid = lanes / 256;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int i = 0; i < 2; i++)
		hipLaunchKernelGGL((k_skel<SIN, SOUT, STAGE, PF>), dim3(grid), dim3(256), 0, 0, src, dst, steps);
	hipEventRecord(a, 0);
	for (int i = 0; i < 20; i++)
		hipLaunchKernelGGL((k_skel<SIN, SOUT, STAGE, PF>), dim3(grid), dim3(256), 0, 0, src, dst, steps);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	ms /= 20;
	const double bytes = (double)lanes * steps * (132 + 256);
	printf("{\"skel\": 1, \"strided_in\": %d, \"strided_out\": %d, \"stage\": %d, \"pf\": %d, \"ms\": %.4f, \"TBs\": %.3f}\n",
	    SIN, SOUT, STAGE, PF, ms, bytes / ms / 1e9);
	hipEventDestroy(a);
	hipEventDestroy(b);
}

/*
 * K1 skeleton with one-eblock groups: a lane consumes 66 B (80-B slot) and
 * emits 128 B per step as two 64-B lines, staged in the consumed buffer
 * (64 x 80 B = 5 KiB per buffer, 10 KiB per wave: four 4-wave workgroups
 * fit a CU).  Lanes/steps chosen by the caller at equal total bytes.
 */
__global__ __launch_bounds__(256) void
k_skel1(const uint8_t *src, uint8_t *dst, uint32_t steps)
{
	constexpr int SEG = 80, NP = 5, LINE = 80, RS = 64 * SEG;
	__shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * RS];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	uint8_t *reg = lds + wv * 2 * RS;
	const uint64_t w = blockIdx.x * 4u + wv;
	const uint32_t CBI = steps * 66u, CBO = steps * 128u;
	uint32_t voff[NP];
#pragma unroll
	for (int i = 0; i < NP; i++) {
		const int k = i * 64 + lane;
		voff[i] = (uint32_t)(k / NP) * CBI + (uint32_t)(k % NP) * 16u;
	}
	const uint8_t *wbi = src + w * 64ull * CBI;
	uint8_t *wbo = dst + w * 64ull * CBO;
	auto issue = [&](uint32_t s, uint8_t *l) {
		const uint8_t *b = wbi + (uint64_t)s * 66u;
#pragma unroll
		for (int i = 0; i < NP; i++)
			dma16(b + voff[i], l + i * 64 * 16);
	};
	issue(0, reg);
	int cur = 0;
	for (uint32_t s = 0; s < steps; s++) {
		uint8_t *cb = reg + (cur ? RS : 0), *ob = reg + (cur ? 0 : RS);
		if (s == 0)
			asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		else
			asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
		uint32_t win[17];
		const uint32_t *m = (const uint32_t *)(cb + lane * SEG);
#pragma unroll
		for (int i = 0; i < 17; i++)
			win[i] = m[i];
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		if (s + 1 < steps)
			issue(s + 1, ob);
		asm volatile("" ::: "memory");
#pragma unroll
		for (int h = 0; h < 2; h++) {
			u32x4 v[4];
#pragma unroll
			for (int q = 0; q < 4; q++)
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const int i = h * 16 + q * 4 + j;
					v[q][j] = win[i % 17] ^ (uint32_t)i;
				}
			uint8_t *line = cb + lane * LINE;
#pragma unroll
			for (int q = 0; q < 4; q++)
				*(u32x4 *)(line + q * 16) = v[q];
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
			/* instruction i: lanes 4k..4k+3 store line 16i+k's pieces */
#pragma unroll
			for (int i = 0; i < 4; i++) {
				const int ln = i * 16 + lane / 4, pc = lane % 4;
				const u32x4 x = *(const u32x4 *)(cb + ln * LINE + pc * 16);
				uint8_t *o = wbo + (uint64_t)ln * CBO + s * 128u + h * 64u + pc * 16u;
				__builtin_nontemporal_store(x, (u32x4 *)o);
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		cur ^= 1;
	}
}

static void
run_skel1(const uint8_t *src, uint8_t *dst, uint32_t lanes, uint32_t steps)
{
	const unsigned grid = lanes / 256;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int i = 0; i < 2; i++)
		hipLaunchKernelGGL(k_skel1, dim3(grid), dim3(256), 0, 0, src, dst, steps);
	hipEventRecord(a, 0);
	for (int i = 0; i < 20; i++)
		hipLaunchKernelGGL(k_skel1, dim3(grid), dim3(256), 0, 0, src, dst, steps);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	ms /= 20;
	const double bytes = (double)grid * 256 * steps * (66 + 128);
	printf("{\"skel1\": 1, \"lanes\": %u, \"steps\": %u, \"wgs\": %u, \"ms\": %.4f, \"TBs\": %.3f}\n",
	    grid * 256, steps, grid, ms, bytes / ms / 1e9);
	hipEventDestroy(a);
	hipEventDestroy(b);
}

/*
 * K1 skeleton with 264-B input runs: a lane's input for two steps (2 x 132
 * B) arrives as one contiguous run, staged half a wave at a time through a
 * single 32 x 272-B landing buffer and kept in VGPRs (two steps ahead), so
 * each DMA instruction reads two ~264-B runs instead of seven 144-B ones.
 * Output staging and stores as k_skel (8.5 + 9 KiB of LDS per wave).
 */
__global__ __launch_bounds__(256) void
k_skel2(const uint8_t *src, uint8_t *dst, uint32_t steps)
{
	constexpr int RUN = 272, HALF = 32 * RUN, NI = (HALF + 1023) / 1024,
	    LINE = 144, OS = 64 * LINE;
	__shared__ __attribute__((aligned(16))) uint8_t lds[4 * (HALF + OS)];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	uint8_t *land = lds + wv * (HALF + OS), *ost = land + HALF;
	const uint64_t w = blockIdx.x * 4u + wv;
	const uint32_t CBI = steps * 132u, CBO = steps * 256u;
	/* piece p of a half-wave landing image: run p / 17, offset p % 17 */
	uint32_t voff[NI];
#pragma unroll
	for (int i = 0; i < NI; i++) {
		const int k = i * 64 + lane;
		voff[i] = (uint32_t)(k / 17) * CBI + (uint32_t)(k % 17) * 16u;
	}
	const uint8_t *wbi = src + w * 64ull * CBI;
	const uint8_t *lim = src + (w + 1) * 64ull * CBI - 16;
	uint8_t *wbo = dst + w * 64ull * CBO;
	/* super-step S covers steps 2S, 2S+1 */
	auto issue = [&](uint32_t S, int h) {
		const uint8_t *b = wbi + (uint64_t)h * 32u * CBI + (uint64_t)S * 264u;
#pragma unroll
		for (int i = 0; i < NI; i++) {
			if (i == NI - 1 && lane >= (HALF / 16) - (NI - 1) * 64)
				break;
			const uint8_t *a = b + voff[i];
			dma16(a < lim ? a : lim, land + i * 1024);
		}
	};
	const uint32_t nS = steps / 2;
	uint32_t cur[66], nxt[66];
	auto take = [&](int h) {
		if ((lane >> 5) == h) {
			const uint32_t *m = (const uint32_t *)(land + (lane & 31) * RUN);
#pragma unroll
			for (int i = 0; i < 66; i++)
				nxt[i] = m[i];
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	};
	/* prologue: super-step 0 into cur */
	issue(0, 0);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	take(0);
	issue(0, 1);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	take(1);
#pragma unroll
	for (int i = 0; i < 66; i++)
		cur[i] = nxt[i];
	if (nS > 1)
		issue(1, 0);
	auto emit = [&](uint32_t s, const uint32_t *win) {
#pragma unroll
		for (int h = 0; h < 2; h++) {
			u32x4 v[8];
#pragma unroll
			for (int q = 0; q < 8; q++)
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const int i = h * 32 + q * 4 + j;
					v[q][j] = win[i % 33] ^ (uint32_t)i;
				}
			uint8_t *line = ost + lane * LINE;
#pragma unroll
			for (int q = 0; q < 8; q++)
				*(u32x4 *)(line + q * 16) = v[q];
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
			for (int i = 0; i < 8; i++) {
				const int ln = i * 8 + lane / 8, pc = lane % 8;
				const u32x4 x = *(const u32x4 *)(ost + ln * LINE + pc * 16);
				uint8_t *o = wbo + (uint64_t)ln * CBO + s * 256u + h * 128u + pc * 16u;
				__builtin_nontemporal_store(x, (u32x4 *)o);
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		}
	};
	for (uint32_t S = 0; S < nS; S++) {
		const bool more = S + 1 < nS;
		if (more) {
			/* first half of S+1 landed (16 stores of step 2S-1 younger) */
			if (S == 0)
				asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
			else
				asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
			take(0);
			issue(S + 1, 1);
		}
		emit(2 * S, cur);
		if (more) {
			asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
			take(1);
			if (S + 2 < nS)
				issue(S + 2, 0);
		}
		emit(2 * S + 1, cur + 33);
#pragma unroll
		for (int i = 0; i < 66; i++)
			cur[i] = nxt[i];
	}
}

static void
run_skel2(const uint8_t *src, uint8_t *dst)
{
	const uint32_t lanes = 125056, steps = 20;
	const unsigned grid = lanes / 256;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int i = 0; i < 2; i++)
		hipLaunchKernelGGL(k_skel2, dim3(grid), dim3(256), 0, 0, src, dst, steps);
	hipEventRecord(a, 0);
	for (int i = 0; i < 20; i++)
		hipLaunchKernelGGL(k_skel2, dim3(grid), dim3(256), 0, 0, src, dst, steps);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	ms /= 20;
	const double bytes = (double)lanes * steps * (132 + 256);
	printf("{\"skel2\": 1, \"run\": 264, \"ms\": %.4f, \"TBs\": %.3f}\n", ms, bytes / ms / 1e9);
	hipEventDestroy(a);
	hipEventDestroy(b);
}

/*
 * Generalised run skeleton: runs of NG groups (NG x 132 B), landed by
 * 64/NG lanes at a time (NG sub-phases per super-step, one group decoded
 * per sub-phase), WPB waves per workgroup and a caller-chosen grid (so the
 * occupancy can drop to one wave per SIMD, where NG = 4 fits the VGPRs).
 */
template <int NG, int WPB>
__global__ __launch_bounds__(64 * WPB, 1) void
k_skelN(const uint8_t *src, uint8_t *dst, uint32_t steps)
{
	constexpr int RUNB = NG * 132, RUN = (RUNB + 15) / 16 * 16, LANES = 64 / NG,
	    IMG = LANES * RUN, NPR = RUN / 16, NI = (LANES * NPR + 63) / 64,
	    LASTL = LANES * NPR - 64 * (NI - 1), LINE = 144, OS = 64 * LINE, RD = NG * 33;
	__shared__ __attribute__((aligned(16))) uint8_t lds[WPB * (IMG + OS)];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	uint8_t *land = lds + wv * (IMG + OS), *ost = land + IMG;
	const uint64_t w = blockIdx.x * (uint64_t)WPB + wv;
	const uint32_t CBI = steps * 132u, CBO = steps * 256u;
	uint32_t voff[NI];
#pragma unroll
	for (int i = 0; i < NI; i++) {
		const int k = i * 64 + lane;
		voff[i] = (uint32_t)(k / NPR) * CBI + (uint32_t)(k % NPR) * 16u;
	}
	const uint8_t *wbi = src + w * 64ull * CBI;
	const uint8_t *lim = src + (w + 1) * 64ull * CBI - 16;
	uint8_t *wbo = dst + w * 64ull * CBO;
	auto issue = [&](uint32_t S, int h) {
		const uint8_t *b = wbi + (uint64_t)h * LANES * CBI + (uint64_t)S * RUNB;
#pragma unroll
		for (int i = 0; i < NI; i++) {
			if (i == NI - 1 && lane >= LASTL)
				break;
			const uint8_t *a = b + voff[i];
			dma16(a < lim ? a : lim, land + i * 1024);
		}
	};
	const uint32_t nS = steps / NG;
	uint32_t A[RD], B[RD];
	auto take = [&](int h, uint32_t *d) {
		if (lane / LANES == h) {
			const uint32_t *m = (const uint32_t *)(land + (lane % LANES) * RUN);
#pragma unroll
			for (int i = 0; i < RD; i++)
				d[i] = m[i];
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	};
	auto emit = [&](uint32_t s, const uint32_t *win) {
#pragma unroll
		for (int h = 0; h < 2; h++) {
			u32x4 v[8];
#pragma unroll
			for (int q = 0; q < 8; q++)
#pragma unroll
				for (int j = 0; j < 4; j++) {
					const int i = h * 32 + q * 4 + j;
					v[q][j] = win[i % 33] ^ (uint32_t)i;
				}
			uint8_t *line = ost + lane * LINE;
#pragma unroll
			for (int q = 0; q < 8; q++)
				*(u32x4 *)(line + q * 16) = v[q];
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
			for (int i = 0; i < 8; i++) {
				const int ln = i * 8 + lane / 8, pc = lane % 8;
				const u32x4 x = *(const u32x4 *)(ost + ln * LINE + pc * 16);
				uint8_t *o = wbo + (uint64_t)ln * CBO + s * 256u + h * 128u + pc * 16u;
				__builtin_nontemporal_store(x, (u32x4 *)o);
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		}
	};
	/* prologue: super-step 0 into A, sub-phase 0 of super-step 1 in flight */
#pragma unroll
	for (int h = 0; h < NG; h++) {
		issue(0, h);
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		take(h, A);
	}
	if (nS > 1)
		issue(1, 0);
	auto step = [&](uint32_t S, uint32_t *cur, uint32_t *nxt) {
		const bool more = S + 1 < nS;
#pragma unroll
		for (int h = 0; h < NG; h++) {
			if (more) {
				if (S == 0 && h == 0)
					asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
				else
					asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
				take(h, nxt);
				if (h + 1 < NG)
					issue(S + 1, h + 1);
				else if (S + 2 < nS)
					issue(S + 2, 0);
			}
			asm volatile("" ::: "memory");
			emit(S * NG + h, cur + h * 33);
		}
	};
	for (uint32_t S = 0; S < nS; S += 2) {
		step(S, A, B);
		if (S + 1 < nS)
			step(S + 1, B, A);
	}
}

template <int NG, int WPB>
static void
run_skelN(const uint8_t *src, uint8_t *dst, uint32_t lanes, uint32_t steps)
{
	const unsigned grid = lanes / (64 * WPB);
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int i = 0; i < 2; i++)
		hipLaunchKernelGGL((k_skelN<NG, WPB>), dim3(grid), dim3(64 * WPB), 0, 0, src, dst, steps);
	hipEventRecord(a, 0);
	for (int i = 0; i < 20; i++)
		hipLaunchKernelGGL((k_skelN<NG, WPB>), dim3(grid), dim3(64 * WPB), 0, 0, src, dst, steps);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	ms /= 20;
	const double bytes = (double)grid * 64 * WPB * steps * (132 + 256);
	printf("{\"skelN\": %d, \"wpb\": %d, \"lanes\": %u, \"steps\": %u, \"wgs\": %u, \"ms\": %.4f, \"TBs\": %.3f}\n",
	    NG, WPB, grid * 64 * WPB, steps, grid, ms, bytes / ms / 1e9);
	hipEventDestroy(a);
	hipEventDestroy(b);
}

int
main()
{
	uint8_t *src;
	uint32_t *sink;
	CHECK(hipMalloc(&src, 400000000));
	CHECK(hipMalloc(&sink, 4));
	CHECK(hipMemset(src, 1, 400000000));
	run<144, 1, false>(src, sink);
	run<144, 2, false>(src, sink);
	run<144, 3, false>(src, sink);
	run<144, 1, true>(src, sink);
	run<144, 2, true>(src, sink);
	run<288, 1, false>(src, sink);
	run<288, 2, false>(src, sink);
	run<528, 1, false>(src, sink);
	run<528, 1, true>(src, sink);
	uint8_t *dst;
	CHECK(hipMalloc(&dst, 700000000));
	run_skel<true, true, true>(src, dst);
	run_skel<true, false, true>(src, dst);
	run_skel<false, true, true>(src, dst);
	run_skel<false, false, true>(src, dst);
	run_skel<true, true, true>(src, dst);
	run_skel2(src, dst);
	run_skelN<2, 4>(src, dst, 125440, 20);
	run_skelN<4, 4>(src, dst, 62720, 40);
	run_skelN<4, 4>(src, dst, 125440, 20);
	run_skelN<2, 4>(src, dst, 62720, 40);
	run_skel2(src, dst);
	CHECK(hipDeviceSynchronize());
	return 0;
}
