/*
 * step_probe.hip -- the predictor step in isolation (registers only, no
 * memory traffic): checks xa_step_lr (packed-f32 stereo step) against the
 * integer xa_step on random and extreme operands, then times both decoding
 * stereo eblocks at 8 waves per CU.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -I bjxa_amd/csrc -o step_probe tools/step_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "xa_common.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ uint32_t
rnd(uint32_t &s)
{
	s = s * 1664525u + 1013904223u;
	return s ^ (s >> 15);
}

/* one step per tuple, both forms; count mismatches */
__global__ void
k_check(uint32_t seed, uint32_t iters, uint32_t *bad)
{
	uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
	uint32_t nbad = 0;
	for (uint32_t i = 0; i < iters; i++) {
		uint32_t r = rnd(s), r2 = rnd(s), r3 = rnd(s);
		/* extremes often: pick from {-32768, 32767, random} */
		int32_t p[4];
		for (int j = 0; j < 4; j++) {
			uint32_t m = (r >> (8 * j)) & 3u;
			uint32_t v = rnd(s);
			p[j] = m == 0 ? -32768 : m == 1 ? 32767 : (int32_t)(int16_t)v;
		}
		const uint32_t gl = r2 % 5u, gr = (r2 >> 8) % 5u;
		const uint32_t rl = (r2 >> 16) & 15u, rr = (r2 >> 20) & 15u;
		const uint32_t cl = r3 & 0xffffu, cr = r3 >> 16;	/* int16 codes */
		int32_t k0l, k1l, k0r, k1r;
		xa_gain(gl, k0l, k1l);
		xa_gain(gr, k0r, k1r);
		int32_t a0 = p[0], a1 = p[1], b0 = p[2], b1 = p[3];
		int32_t sl = xa_step((int32_t)(cl << 16), 16u + rl, k0l, k1l, a0, a1);
		int32_t sr = xa_step((int32_t)(cr << 16), 16u + rr, k0r, k1r, b0, b1);
		const uint32_t want = ((uint32_t)sl & 0xffffu) | ((uint32_t)sr << 16);
		float f0l, f1l, f0r, f1r;
		xa_gain_f(gl, f0l, f1l);
		xa_gain_f(gr, f0r, f1r);
		xa_f2 q0 = {(float)p[0], (float)p[2]}, q1 = {(float)p[1], (float)p[3]};
		const uint32_t t = xa_pk_ashr(cl | (cr << 16), rl | (rr << 16));
		const uint32_t got = xa_step_lr(t, xa_f2{f0l, f0r}, xa_f2{f1l, f1r},
		    q0, q1);
		nbad += (got != want) || ((int32_t)q0.x != sl) ||
		    ((int32_t)q0.y != sr) || ((int32_t)q1.x != p[0]) ||
		    ((int32_t)q1.y != p[2]);
	}
	if (nbad)
		atomicAdd(bad, nbad);
}

/* decode `neb` stereo eblocks of register-generated codes per lane; both
 * forms fold their frames into a checksum */
template <bool LR>
__global__ __launch_bounds__(256) void
k_time(uint32_t seed, uint32_t neb, uint32_t *out)
{
	uint32_t s = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
	int32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
	xa_f2 q0 = {0.f, 0.f}, q1 = {0.f, 0.f};
	uint32_t acc = 0;
	for (uint32_t e = 0; e < neb; e++) {
		const uint32_t prof = rnd(s);
		const uint32_t gl = (prof & 0xffu) % 5u, gr = ((prof >> 8) & 0xffu) % 5u;
		const uint32_t rl = (prof >> 16) & 15u, rr = (prof >> 20) & 15u;
		uint32_t wl[8], wr[8];
#pragma unroll
		for (int i = 0; i < 8; i++) {
			wl[i] = rnd(s);
			wr[i] = wl[i] * 0x9e3779b9u;
		}
		if (LR) {
			float f0l, f1l, f0r, f1r;
			xa_gain_f(gl, f0l, f1l);
			xa_gain_f(gr, f0r, f1r);
			const xa_f2 k0 = {f0l, f0r}, k1 = {f1l, f1r};
			const uint32_t sh = rl | (rr << 16);
#pragma unroll
			for (int n = 0; n < 32; n++) {
				/* bytes n of both blocks into the high bytes of the
				 * halves: L -> bits 8..15, R -> bits 24..31 */
				const uint32_t sel = 0x000c000cu | (uint32_t)(n & 3) << 8 |
				    (uint32_t)(4 + (n & 3)) << 24;
				const uint32_t tp = __builtin_amdgcn_perm(wr[n >> 2],
				    wl[n >> 2], sel);
				acc += xa_step_lr(xa_pk_ashr(tp, sh), k0, k1, q0, q1);
			}
		} else {
			int32_t k0l, k1l, k0r, k1r;
			xa_gain(gl, k0l, k1l);
			xa_gain(gr, k0r, k1r);
#pragma unroll
			for (int n = 0; n < 32; n++) {
				const uint32_t sel = 0x000c0c0cu | (uint32_t)(n & 3) << 24;
				int32_t sl = xa_step((int32_t)__builtin_amdgcn_perm(0u,
				    wl[n >> 2], sel), 16u + rl, k0l, k1l, a0, a1);
				int32_t sr = xa_step((int32_t)__builtin_amdgcn_perm(0u,
				    wr[n >> 2], sel), 16u + rr, k0r, k1r, b0, b1);
				acc += __builtin_amdgcn_perm((uint32_t)sr, (uint32_t)sl,
				    0x05040100u);
			}
		}
	}
	out[blockIdx.x * 256 + threadIdx.x] = acc;
}


/* dependent-chain latency: one wave per CU, every lane runs one chain of
 * 32*nblk samples (codes from registers); cycles per sample from
 * s_memtime around the loop.  V: 0 xa_step, 1 repair step (4-op chain),
 * 2 xa_step_f, 3 xa_step_lr (per frame = two chains) */
__device__ __forceinline__ int32_t
lat_step(int32_t top, uint32_t sh, int32_t k0, int32_t k1, int32_t &p0, int32_t &p1)
{
	const int32_t t256 = (top >> sh) << 8;
	const int32_t c = __mul24(p1, k1) + t256;
	const int32_t ha = __mul24(p0, k0) + c;
	const int32_t hb = __mul24(p0, k0) + (c + 255);
	const int32_t s = __builtin_amdgcn_fmed3f(0, 0, 0) == 0.f ?
	    max(min(min(ha, 32767 * 256 + 255), max(hb, -32768 * 256)),
	    min(max(min(ha, 32767 * 256 + 255), max(hb, -32768 * 256)), t256)) >> 8 : 0;
	p1 = p0;
	p0 = s;
	return s;
}

template <int V>
__global__ __launch_bounds__(64) void
k_lat(uint32_t seed, uint32_t nblk, uint32_t *out, uint64_t *cyc)
{
	uint32_t s = seed ^ threadIdx.x * 2654435761u;
	int32_t a0 = 0, a1 = 0;
	float f0 = 0.f, f1 = 0.f;
	xa_f2 q0 = {0.f, 0.f}, q1 = {0.f, 0.f};
	uint32_t acc = 0;
	const uint64_t t0 = __builtin_amdgcn_s_memtime();
	for (uint32_t e = 0; e < nblk; e++) {
		const uint32_t prof = rnd(s);
		const uint32_t g = (prof & 0xffu) % 5u, r = (prof >> 16) & 15u;
		int32_t k0, k1;
		xa_gain(g, k0, k1);
		float fk0, fk1;
		xa_gain_f(g, fk0, fk1);
		uint32_t wl[8];
#pragma unroll
		for (int i = 0; i < 8; i++)
			wl[i] = rnd(s);
#pragma unroll
		for (int n = 0; n < 32; n += 2) {
			const uint32_t sel = 0x000c0c0cu | (uint32_t)(n & 3) << 24;
			const int32_t ta = (int32_t)__builtin_amdgcn_perm(0u, wl[n >> 2], sel);
			const int32_t tb = (int32_t)__builtin_amdgcn_perm(0u, wl[n >> 2], sel + (1u << 24));
			if (V == 0) {
				acc += xa_step(ta, 16u + r, k0, k1, a0, a1);
				acc += xa_step(tb, 16u + r, k0, k1, a0, a1);
			} else if (V == 1) {
				acc += lat_step(ta, 16u + r, k0, k1, a0, a1);
				acc += lat_step(tb, 16u + r, k0, k1, a0, a1);
			} else if (V == 2) {
				const uint32_t t = xa_pk_ashr(((uint32_t)ta >> 16) | ((uint32_t)tb & 0xffff0000u), r | r << 16);
				acc += xa_step_f<false>(t, fk0, fk1, f0, f1);
				acc += xa_step_f<true>(t, fk0, fk1, f0, f1);
			} else {
				const uint32_t t = xa_pk_ashr(((uint32_t)ta >> 16) | ((uint32_t)tb & 0xffff0000u), r | r << 16);
				acc += xa_step_lr(t, xa_f2{fk0, fk0}, xa_f2{fk1, fk1}, q0, q1);
			}
		}
	}
	const uint64_t t1 = __builtin_amdgcn_s_memtime();
	out[blockIdx.x * 64 + threadIdx.x] = acc;
	if (threadIdx.x == 0)
		cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static double
lat_run(uint32_t *o, uint64_t *c)
{
	const uint32_t nblk = 256;
	hipLaunchKernelGGL((k_lat<V>), dim3(256), dim3(64), 0, 0, 3u, nblk, o, c);
	hipLaunchKernelGGL((k_lat<V>), dim3(256), dim3(64), 0, 0, 3u, nblk, o, c);
	hipDeviceSynchronize();
	static uint64_t h[256];
	hipMemcpy(h, c, sizeof h, hipMemcpyDeviceToHost);
	double m = 0;
	for (int i = 0; i < 256; i++)
		m += (double)h[i];
	m /= 256;
	/* samples per lane: 32 per block (V 3: 16 frames = 32 samples) */
	return m / (nblk * 32.0);
}

int
main()
{
	uint32_t *bad, *o1, *o2;
	const unsigned grid = 2048 * 64 / 256;	/* 8 waves per CU */
	CHECK(hipMalloc(&bad, 4));
	CHECK(hipMalloc(&o1, grid * 256 * 4));
	CHECK(hipMalloc(&o2, grid * 256 * 4));
	CHECK(hipMemset(bad, 0, 4));
	k_check<<<1024, 256>>>(12345u, 1024, bad);
	uint32_t nb = 0;
	CHECK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
	printf("{\"check_tuples\": %u, \"mismatches\": %u}\n", 1024u * 256u * 1024u, nb);

	const uint32_t neb = 48;
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	float ms[2];
	for (int v = 0; v < 2; v++) {
		for (int i = 0; i < 3; i++) {
			if (v) k_time<true><<<grid, 256>>>(7u, neb, o2);
			else k_time<false><<<grid, 256>>>(7u, neb, o1);
		}
		hipEventRecord(a, 0);
		for (int i = 0; i < 10; i++) {
			if (v) k_time<true><<<grid, 256>>>(7u, neb, o2);
			else k_time<false><<<grid, 256>>>(7u, neb, o1);
		}
		hipEventRecord(b, 0);
		hipEventSynchronize(b);
		hipEventElapsedTime(&ms[v], a, b);
		ms[v] /= 10;
	}
	static uint32_t h1[grid * 256], h2[grid * 256];
	CHECK(hipMemcpy(h1, o1, sizeof h1, hipMemcpyDeviceToHost));
	CHECK(hipMemcpy(h2, o2, sizeof h2, hipMemcpyDeviceToHost));
	unsigned diff = 0;
	for (unsigned i = 0; i < grid * 256; i++)
		diff += h1[i] != h2[i];
	/* per-wave cycles per stereo sample pair at ~2.1 GHz is ms * 2.1e6 /
	 * (neb * 32) per wave-slot pair; report ns per frame per lane-slot */
	printf("{\"int_ms\": %.4f, \"lr_ms\": %.4f, \"lanes_differ\": %u, "
	    "\"int_ns_per_frame_wave\": %.3f, \"lr_ns_per_frame_wave\": %.3f}\n",
	    ms[0], ms[1], diff, ms[0] * 1e6 / (neb * 32) / 2, ms[1] * 1e6 / (neb * 32) / 2);
	uint64_t *cy;
	CHECK(hipMalloc(&cy, 256 * 8));
	printf("{\"memtime_ticks_per_sample\": {\"int\": %.2f, \"repair\": %.2f, \"f32\": %.2f, \"lr_per_2\": %.2f}}\n",
	    lat_run<0>(o1, cy), lat_run<1>(o1, cy), lat_run<2>(o1, cy), lat_run<3>(o1, cy));
	return 0;
}
