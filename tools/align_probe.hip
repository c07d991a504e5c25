/*
 * align_probe.hip -- does K1's input pattern pay for runs that straddle
 * 128-B lines?  The k_skel2 skeleton of pattern_probe.hip (a lane's input
 * for a super-step is one contiguous run, landed half a wave at a time by
 * LDS-DMA, kept in VGPRs; output staged in LDS and stored 8 whole lines per
 * instruction) with the run length RUNB, the lane stride and a base offset
 * as parameters:
 *   264 B runs at a 2640-B lane stride   (K1 on C3: runs start anywhere)
 *   256 B runs at a 2560-B stride, base 0 (every run two whole lines)
 *   256 B runs, base 64 / base 8          (same bytes, straddling lines)
 *   384 B runs at a 3840-B stride, base 0 (three whole lines)
 * Prints JSON lines (ms, TB/s of in+out bytes).
 *
 * build: hipcc --offload-arch=gfx950 -O3 -o align_probe tools/align_probe.hip
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

/* RUNB bytes per lane per super-step (two output steps of 256 B each) */
template <int RUNB, bool LINES = false>
__global__ __launch_bounds__(256, 2) void
k_run(const uint8_t *src, uint8_t *dst, uint32_t nS)
{
	/* LINES: land the 3 whole 128-B lines that cover each run (384 B) and
	 * stage the output unpadded (128-B lines), 20 KiB per wave */
	constexpr int RUN = LINES ? 384 : (RUNB + 15) / 16 * 16, NPR = RUN / 16,
	    HALF = 32 * RUN, NI = (32 * NPR + 63) / 64, LASTL = 32 * NPR - 64 * (NI - 1),
	    RD = RUNB / 4, LINE = LINES ? 128 : 144, OS = 64 * LINE;
	__shared__ __attribute__((aligned(16))) uint8_t lds[4 * (HALF + OS)];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	uint8_t *land = lds + wv * (HALF + OS), *ost = land + HALF;
	const uint64_t w = blockIdx.x * 4u + wv;
	const uint32_t CBI = nS * RUNB, CBO = nS * 512u;
	uint32_t voff[NI];
#pragma unroll
	for (int i = 0; i < NI; i++) {
		const int k = i * 64 + lane;
		voff[i] = (uint32_t)(k / NPR) * CBI + (uint32_t)(k % NPR) * 16u;
	}
	const uint8_t *wbi = src + w * 64ull * CBI;
	uint8_t *wbo = dst + w * 64ull * CBO;
	auto issue = [&](uint32_t S, int h) {
		const uint8_t *b = wbi + (uint64_t)h * 32u * CBI + (uint64_t)S * RUNB;
#pragma unroll
		for (int i = 0; i < NI; i++) {
			if (i == NI - 1 && lane >= LASTL)
				break;
			const uint8_t *a = b + voff[i];
			if (LINES) {
				/* piece k of run r: the line-aligned base of run r */
				const int k = i * 64 + lane, r = k / NPR, pc = k % NPR;
				const uint8_t *rb = b + (uint64_t)r * CBI;
				a = (const uint8_t *)((uintptr_t)rb & ~(uintptr_t)127) + pc * 16;
			}
			dma16(a, land + i * 1024);
		}
	};
	uint32_t cur[RD], nxt[RD];
	auto take = [&](int h) {
		if ((lane >> 5) == h) {
			const uint32_t *m = (const uint32_t *)(land + (lane & 31) * RUN +
			    (LINES ? (((uintptr_t)wbi + (uint64_t)(lane >> 5) * 32u * CBI +
			    (uint64_t)(lane & 31) * CBI) & 127) : 0));
#pragma unroll
			for (int i = 0; i < RD; i++)
				nxt[i] = m[i];
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	};
	issue(0, 0);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	take(0);
	issue(0, 1);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	take(1);
#pragma unroll
	for (int i = 0; i < RD; i++)
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
					v[q][j] = win[i % (RD / 2)] ^ (uint32_t)i;
				}
			uint8_t *line = ost + lane * LINE;
#pragma unroll
			for (int q = 0; q < 8; q++)
				*(u32x4 *)(line + 16 * (LINES ? (q ^ (lane & 7)) : q)) = v[q];
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
			for (int i = 0; i < 8; i++) {
				const int ln = i * 8 + lane / 8, pc = lane % 8;
				const u32x4 x = *(const u32x4 *)(ost + ln * LINE +
				    16 * (LINES ? (pc ^ (ln & 7)) : pc));
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
		emit(2 * S + 1, cur + RD / 2);
#pragma unroll
		for (int i = 0; i < RD; i++)
			cur[i] = nxt[i];
	}
}

/*
 * The byte-stream structure K1 would need for line-exact input: each lane's
 * landing slot is [carry line | 2 new lines] (384 B); a super-step DMAs only
 * the 2 new whole lines of every run (pieces that would land in a carry
 * area are masked off: 12 instructions per half instead of 8), the lane
 * reads its 264-B run from the slot at its own byte offset, then copies the
 * slot's last line into the carry area for the next super-step.  Output
 * staged unpadded with an XOR swizzle (8 KiB per wave).  Source: 256 new
 * bytes per lane per super-step (two aligned lines), lane stride nS*256.
 */
__global__ __launch_bounds__(256, 2) void
k_carry(const uint8_t *src, uint8_t *dst, uint32_t nS)
{
	constexpr int SLOT = 384, HALF = 32 * SLOT, NI = HALF / 1024, RD = 66,
	    LINE = 128, OS = 64 * LINE;
	__shared__ __attribute__((aligned(16))) uint8_t lds[4 * (HALF + OS)];
	const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	uint8_t *land = lds + wv * (HALF + OS), *ost = land + HALF;
	const uint64_t w = blockIdx.x * 4u + wv;
	const uint32_t CBI = nS * 256u, CBO = nS * 512u;
	uint32_t voff[NI];
	bool von[NI];
#pragma unroll
	for (int i = 0; i < NI; i++) {
		const int k = i * 64 + lane, r = k / 24, pc = k % 24;
		von[i] = pc >= 8;
		voff[i] = (uint32_t)r * CBI + (uint32_t)(pc >= 8 ? pc - 8 : 0) * 16u;
	}
	const uint8_t *wbi = src + w * 64ull * CBI;
	uint8_t *wbo = dst + w * 64ull * CBO;
	const int o = (lane * 8) & 120;		/* a run's byte offset in its slot */
	auto issue = [&](uint32_t S, int h) {
		const uint8_t *b = wbi + (uint64_t)h * 32u * CBI + (uint64_t)S * 256u;
#pragma unroll
		for (int i = 0; i < NI; i++)
			if (von[i])
				dma16(b + voff[i], land + i * 1024);
	};
	uint32_t cur[RD], nxt[RD];
	auto take = [&](int h) {
		if ((lane >> 5) == h) {
			uint8_t *sl = land + (lane & 31) * SLOT;
			const uint32_t *m = (const uint32_t *)(sl + o);
#pragma unroll
			for (int i = 0; i < RD; i++)
				nxt[i] = m[i];
			u32x4 c[8];
#pragma unroll
			for (int i = 0; i < 8; i++)
				c[i] = *(const u32x4 *)(sl + 256 + 16 * i);
#pragma unroll
			for (int i = 0; i < 8; i++)
				*(u32x4 *)(sl + 16 * i) = c[i];
		}
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	};
	issue(0, 0);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	take(0);
	issue(0, 1);
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	take(1);
#pragma unroll
	for (int i = 0; i < RD; i++)
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
				*(u32x4 *)(line + 16 * (q ^ (lane & 7))) = v[q];
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
			for (int i = 0; i < 8; i++) {
				const int ln = i * 8 + lane / 8, pc = lane % 8;
				const u32x4 x = *(const u32x4 *)(ost + ln * LINE + 16 * (pc ^ (ln & 7)));
				uint8_t *op = wbo + (uint64_t)ln * CBO + s * 256u + h * 128u + pc * 16u;
				__builtin_nontemporal_store(x, (u32x4 *)op);
			}
			__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
			__builtin_amdgcn_wave_barrier();
			__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
		}
	};
	for (uint32_t S = 0; S < nS; S++) {
		const bool more = S + 1 < nS;
		if (more) {
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
		for (int i = 0; i < RD; i++)
			cur[i] = nxt[i];
	}
}

static void
run_carry(const uint8_t *src, uint8_t *dst, uint32_t nS)
{
	const uint32_t lanes = 125440;
	const unsigned grid = lanes / 256;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int i = 0; i < 2; i++)
		hipLaunchKernelGGL(k_carry, dim3(grid), dim3(256), 0, 0, src, dst, nS);
	hipEventRecord(a, 0);
	for (int i = 0; i < 20; i++)
		hipLaunchKernelGGL(k_carry, dim3(grid), dim3(256), 0, 0, src, dst, nS);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	ms /= 20;
	const double bytes = (double)lanes * nS * (256 + 512);
	printf("{\"case\": \"carry line + 2 new lines\", \"supersteps\": %u, \"ms\": %.4f, \"TBs\": %.3f}\n",
	    nS, ms, bytes / ms / 1e9);
	hipEventDestroy(a);
	hipEventDestroy(b);
}

template <int RUNB, bool LINES = false>
static void
run(const uint8_t *src, uint8_t *dst, uint32_t base, uint32_t nS, const char *tag)
{
	const uint32_t lanes = 125440;
	const unsigned grid = lanes / 256;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	for (int i = 0; i < 2; i++)
		hipLaunchKernelGGL((k_run<RUNB, LINES>), dim3(grid), dim3(256), 0, 0, src + base, dst, nS);
	hipEventRecord(a, 0);
	for (int i = 0; i < 20; i++)
		hipLaunchKernelGGL((k_run<RUNB, LINES>), dim3(grid), dim3(256), 0, 0, src + base, dst, nS);
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	ms /= 20;
	const double bytes = (double)lanes * nS * (RUNB + 512);
	printf("{\"case\": \"%s\", \"run\": %d, \"base\": %u, \"supersteps\": %u, \"pcm_stride\": %u, \"ms\": %.4f, \"TBs\": %.3f}\n",
	    tag, RUNB, base, nS, nS * 512u, ms, bytes / ms / 1e9);
	hipEventDestroy(a);
	hipEventDestroy(b);
}

int
main(int argc, char **argv)
{
	uint8_t *src, *dst;
	if (argc > 1 && argv[1][0] == 'r') {
		/* does the rate depend on where dst lies relative to src?  six
		 * fresh buffer pairs (dst 2 MiB oversized), each timed with dst
		 * shifted by 0 .. 1 MiB inside its allocation */
		const size_t ni = 125440ull * 264 * 10, no = 125440ull * 512 * 10;
		const size_t sh[] = {0, 2048, 4096, 8192, 16384, 65536, 262144, 1048576};
		for (int k = 0; k < 6; k++) {
			uint8_t *sk, *dk;
			CHECK(hipMalloc(&sk, ni));
			CHECK(hipMalloc(&dk, no + (2u << 20)));
			CHECK(hipMemset(sk, 1, ni));
			if (k == 3) {
				uint8_t *d;
				CHECK(hipMalloc(&d, 16ull << 30));
			}
			printf("{\"pair\": %d, \"src\": \"%p\", \"dst\": \"%p\"}\n", k, sk, dk);
			for (size_t o : sh) {
				char t[64];
				snprintf(t, sizeof t, "pair %d dst+%zu", k, o);
				run<264>(sk, dk + o, 0, 10, t);
			}
		}
		return 0;
	}
	if (argc > 1 && argv[1][0] == 'q') {
		/* placement, finer: exact-size buffer pairs allocated after 0, 1,
		 * 4, 16 and 64 GiB of other allocations (all kept), timed
		 * interleaved */
		const size_t ni = 125440ull * 264 * 10, no = 125440ull * 512 * 10;
		const size_t pad[] = {0, 1ull << 30, 3ull << 30, 12ull << 30, 48ull << 30};
		const char *tag[] = {"after 0 GiB", "after 1 GiB", "after 4 GiB", "after 16 GiB", "after 64 GiB"};
		uint8_t *si[5], *di[5];
		for (int k = 0; k < 5; k++) {
			if (pad[k]) {
				uint8_t *d;
				CHECK(hipMalloc(&d, pad[k]));
			}
			CHECK(hipMalloc(&si[k], ni));
			CHECK(hipMalloc(&di[k], no));
			CHECK(hipMemset(si[k], 1, ni));
			CHECK(hipMemset(di[k], 0, no));
			printf("{\"alloc\": \"%s\", \"src\": \"%p\", \"dst\": \"%p\"}\n", tag[k], si[k], di[k]);
		}
		for (int rep = 0; rep < 3; rep++)
			for (int k = 0; k < 5; k++)
				run<264>(si[k], di[k], 0, 10, tag[k]);
		return 0;
	}
	if (argc > 1 && argv[1][0] == 'p') {
		/* placement: the C3 pattern (nS = 10) on buffers allocated in
		 * different ways */
		const size_t ni = 125440ull * 264 * 10, no = 125440ull * 512 * 10;
		uint8_t *s1, *d1, *big, *s3, *d3, *dummy, *s4, *d4;
		CHECK(hipMalloc(&s1, ni));
		CHECK(hipMalloc(&d1, no));
		CHECK(hipMalloc(&big, 4ull << 30));
		CHECK(hipMalloc(&s3, 125440ull * 264 * 128));
		CHECK(hipMalloc(&d3, 125440ull * 512 * 128));
		CHECK(hipMalloc(&dummy, 16ull << 30));
		CHECK(hipMalloc(&s4, ni));
		CHECK(hipMalloc(&d4, no));
		CHECK(hipMemset(s1, 1, ni));
		CHECK(hipMemset(big, 1, 4ull << 30));
		CHECK(hipMemset(s3, 1, ni));
		CHECK(hipMemset(s4, 1, ni));
		printf("{\"ptrs\": [\"%p\", \"%p\", \"%p\", \"%p\", \"%p\", \"%p\", \"%p\"]}\n",
		    s1, d1, big, s3, d3, s4, d4);
		for (int rep = 0; rep < 3; rep++) {
			run<264>(s1, d1, 0, 10, "exact-size buffers");
			run<264>(big, big + (1ull << 30), 0, 10, "one 4 GiB buffer");
			run<264>(s3, d3, 0, 10, "4 / 8 GB buffers");
			run<264>(s4, d4, 0, 10, "exact-size after a 16 GiB buffer");
			run<264>(big + (2ull << 20), big + (1ull << 30) + (6ull << 20), 0, 10, "4 GiB buffer, +2/+6 MiB");
		}
		return 0;
	}
	if (argc > 1) {
		/* lane-stride sweep: K1's C3 pattern (264-B runs, 4 eblocks per
		 * super-step) with nS super-steps per lane, i.e. chunks of 4 nS
		 * eblocks at an input stride of 264 nS and a PCM stride of 512 nS
		 * bytes, on a chip-filling grid */
		const uint32_t ns[] = {8, 10, 12, 14, 15, 16, 17, 18, 20, 24, 30, 31, 32, 33, 48, 64, 65, 128};
		CHECK(hipMalloc(&src, 125440ull * 264 * 128 + 4096));
		CHECK(hipMalloc(&dst, 125440ull * 512 * 128 + 4096));
		CHECK(hipMemset(src, 1, 125440ull * 264 * 128));
		for (int rep = 0; rep < 2; rep++)
			for (uint32_t n : ns)
				run<264>(src, dst, 0, n, "stride sweep");
		return 0;
	}
	CHECK(hipMalloc(&src, 500000000));
	CHECK(hipMalloc(&dst, 700000000));
	CHECK(hipMemset(src, 1, 500000000));
	for (int rep = 0; rep < 2; rep++) {
		run<264>(src, dst, 0, 10, "K1 C3 runs");
		run<256>(src, dst, 0, 10, "two whole lines");
		run<256>(src, dst, 64, 10, "256 at +64");
		run<256>(src, dst, 8, 10, "256 at +8");
		run<264>(src, dst, 120, 10, "264 at +120");
		run<256>(src, dst, 0, 10, "two whole lines");
		run<264, true>(src, dst, 0, 10, "264 via 3 whole lines");
		run<264, true>(src, dst, 120, 10, "264 via 3 whole lines, +120");
		run_carry(src, dst, 10);
	}
	CHECK(hipDeviceSynchronize());
	return 0;
}
