/*
 * rdreq_calib.hip -- what one TCC_EA0_RDREQ is worth, on known byte counts.
 *
 * MI355X_MICROARCH.md §HBM: FETCH_SIZE is calibrated only for 16-B/lane
 * streaming reads (it reports half of them); the derived FETCH_SIZE of
 * rocprofv3 is TCC_BUBBLE x 128 + (RDREQ - BUBBLE - RDREQ_32B) x 64 +
 * RDREQ_32B x 32.  This probe reads buffers far larger than the 256 MiB
 * Infinity Cache with the load forms and patterns the decode uses, each
 * kernel reading a byte count known exactly, so that the counters of one
 * rocprofv3 --pmc pass give bytes per request for each form:
 *
 *   k_vec        contiguous global_load_dwordx4 (the guide's calibrated case)
 *   k_dma16      contiguous LDS-DMA, 16 B per lane (1 KiB per instruction)
 *   k_dma4       contiguous LDS-DMA, 4 B per lane
 *   k_runs<264>  K1's input pattern on C3: lane l of a wave reads runs of
 *                264 B (landed as 17 16-B pieces, half a wave per buffer)
 *                at a 2,640-B lane stride, 10 runs per lane, consecutive
 *                runs of a lane contiguous -- every byte of the buffer is
 *                read once, 8 B of each run twice (the 272-B rounding;
 *                the buffer has 4 KiB of slack past the last run)
 *   k_runs<256>  the same with 256-B runs at a 2,560-B stride, base 0:
 *                every run is two whole 128-B lines
 *   k_vec (small) a 96 MiB buffer read twice back to back: the second
 *                launch is served by the Infinity Cache, which shows whether
 *                its hits are counted
 * Each kernel is launched 3 times (the counters are per dispatch).  Prints
 * one JSON line: bytes and event ms per kernel.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -o rdreq_calib tools/rdreq_calib.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define LDS_PTR(p) ((__attribute__((address_space(3))) void *)(p))
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(256) void
k_vec(const u32x4 *__restrict__ in, uint32_t *sink, size_t n)
{
	uint32_t acc = 0;
	for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n;
	    i += (size_t)gridDim.x * 256) {
		u32x4 v = in[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x12345678u)
		*sink = acc;
}

/* contiguous LDS-DMA: each wave instruction lands PS x 64 bytes */
template <int PS>
__global__ __launch_bounds__(256) void
k_dma(const uint8_t *__restrict__ in, uint32_t *sink, size_t nbytes)
{
	__shared__ __attribute__((aligned(16))) uint8_t lds[4][8 * 64 * PS];
	const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
	constexpr size_t WI = 64 * PS;			/* bytes per instruction */
	const size_t nw = (size_t)gridDim.x * 4;
	size_t w = (size_t)blockIdx.x * 4 + wv;
	int slot = 0;
	for (size_t off = w * 8 * WI; off < nbytes; off += nw * 8 * WI) {
#pragma unroll
		for (int u = 0; u < 8; u++) {
			const size_t o = off + u * WI;
			if (o + WI > nbytes)
				continue;
			if constexpr (PS == 16)
				__builtin_amdgcn_global_load_lds(in + o + lane * PS,
				    LDS_PTR(&lds[wv][u * WI]), 16, 0, 0);
			else
				__builtin_amdgcn_global_load_lds(in + o + lane * PS,
				    LDS_PTR(&lds[wv][u * WI]), 4, 0, 0);
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		slot ^= 1;
	}
	__syncthreads();
	if (lds[wv][lane] == 0xee && lds[wv][lane + 1] == 0x12)
		*sink = slot;
}

/* (the builtin inside a kernel template loses the host stub; wrap it) */
__device__ __forceinline__ void
dma16(const void *g, uint8_t *l)
{
	__builtin_amdgcn_global_load_lds(g, LDS_PTR(l), 16, 0, 0);
}

/* K1's input pattern (no decode, no stores): RUNB bytes per lane per step,
 * nS steps, lanes of a wave at stride nS * RUNB, landed half a wave at a
 * time in 16-B pieces (RUNB rounded up to 16 B) */
template <int RUNB>
__global__ __launch_bounds__(256) void
k_runs(const uint8_t *__restrict__ src, uint32_t *sink, uint32_t nS)
{
	constexpr int RUN = (RUNB + 15) / 16 * 16, NPR = RUN / 16, HALF = 32 * RUN,
	    NI = (32 * NPR + 63) / 64, LASTL = 32 * NPR - 64 * (NI - 1);
	__shared__ __attribute__((aligned(16))) uint8_t lds[4 * 2 * HALF];
	const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
	uint8_t *land = lds + wv * 2 * HALF;
	const uint64_t w = blockIdx.x * 4u + wv;
	const uint32_t CBI = nS * RUNB;
	uint32_t voff[NI];
#pragma unroll
	for (int i = 0; i < NI; i++) {
		const int k = i * 64 + lane;
		voff[i] = (uint32_t)(k / NPR) * CBI + (uint32_t)(k % NPR) * 16u;
	}
	const uint8_t *wbi = src + w * 64ull * CBI;
	uint32_t acc = 0;
	for (uint32_t S = 0; S < nS; S++) {
#pragma unroll
		for (int h = 0; h < 2; h++) {
			const uint8_t *b = wbi + (uint64_t)h * 32u * CBI + (uint64_t)S * RUNB;
#pragma unroll
			for (int i = 0; i < NI; i++) {
				if (i == NI - 1 && lane >= LASTL)
					break;
				dma16(b + voff[i], land + h * HALF + i * 1024);
			}
		}
		asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
		acc ^= *(const uint32_t *)(land + lane * 16);
	}
	if (acc == 0x12345678u)
		*sink = acc;
}

/* launched only from lambdas: instantiate the stubs explicitly */
template __global__ void k_runs<264>(const uint8_t *, uint32_t *, uint32_t);
template __global__ void k_runs<256>(const uint8_t *, uint32_t *, uint32_t);
template __global__ void k_dma<16>(const uint8_t *, uint32_t *, size_t);
template __global__ void k_dma<4>(const uint8_t *, uint32_t *, size_t);

template <typename F>
static float
time3(F f)
{
	hipEvent_t a, b;
	(void)hipEventCreate(&a);
	(void)hipEventCreate(&b);
	float best = 1e9f;
	for (int i = 0; i < 3; i++) {
		(void)hipEventRecord(a, 0);
		f();
		(void)hipEventRecord(b, 0);
		(void)hipEventSynchronize(b);
		float ms;
		(void)hipEventElapsedTime(&ms, a, b);
		best = ms < best ? ms : best;
	}
	(void)hipEventDestroy(a);
	(void)hipEventDestroy(b);
	return best;
}

int
main()
{
	/* 1.32 GB: K1's C3 pattern (1,953 waves of 64 lanes x 2,640 B) x 4 */
	const uint32_t nS = 10, waves = 4 * 1952;
	const size_t R264 = (size_t)waves * 64 * nS * 264;
	const size_t R256 = (size_t)waves * 64 * nS * 256;
	const size_t SMALL = 96ull << 20;
	uint8_t *in;
	uint32_t *sink;
	CHECK(hipMalloc(&in, R264 + 4096));
	CHECK(hipMalloc(&sink, 4));
	CHECK(hipMemset(in, 1, R264 + 4096));
	CHECK(hipDeviceSynchronize());
	const size_t R = R256;		/* contiguous kernels: 1.28 GB */
	float t_vec = time3([&] { k_vec<<<2048, 256>>>((const u32x4 *)in, sink, R / 16); });
	float t_d16 = time3([&] { k_dma<16><<<2048, 256>>>(in, sink, R); });
	float t_d4 = time3([&] { k_dma<4><<<2048, 256>>>(in, sink, R); });
	float t_r264 = time3([&] { k_runs<264><<<waves / 4, 256>>>(in, sink, nS); });
	float t_r256 = time3([&] { k_runs<256><<<waves / 4, 256>>>(in, sink, nS); });
	/* Infinity-Cache test: 96 MiB read 3 times back to back (the first
	 * launch of time3 fills the cache, the next two hit it) */
	float t_small = time3([&] { k_vec<<<2048, 256>>>((const u32x4 *)in, sink, SMALL / 16); });
	CHECK(hipDeviceSynchronize());
	printf("{\"vec_bytes\": %zu, \"vec_ms\": %.4f, \"dma16_bytes\": %zu, \"dma16_ms\": %.4f, "
	    "\"dma4_bytes\": %zu, \"dma4_ms\": %.4f, \"runs264_bytes\": %zu, \"runs264_ms\": %.4f, "
	    "\"runs256_bytes\": %zu, \"runs256_ms\": %.4f, \"small_bytes\": %zu, \"small_ms\": %.4f}\n",
	    R, t_vec, R, t_d16, R, t_d4, R264, t_r264, R256, t_r256, SMALL, t_small);
	return 0;
}
