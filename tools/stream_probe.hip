/*
 * stream_probe.hip -- practical HBM ceilings for the decode's traffic shape,
 * with hand-written streaming kernels (not torch ops):
 *   expand  read R bytes, write 2R (each 16-B piece read once, written as
 *           two 16-B pieces of the output, non-temporal), contiguous
 *   read    read-only sum of R bytes
 *   write   write-only fill of 2R bytes (non-temporal)
 *   copy    1:1 copy of R bytes
 * Each kernel is timed with hipEvents over 20 launches; R = 330 MB (the C3
 * stream), output 660 MB.  Prints one JSON line.
 *
 * build: hipcc --offload-arch=gfx950 -O3 -o stream_probe tools/stream_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int U>
__global__ __launch_bounds__(256) void
k_expand(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n)
{
	size_t i = ((size_t)blockIdx.x * 256 * U) + threadIdx.x;
	u32x4 v[U];
#pragma unroll
	for (int u = 0; u < U; u++)
		v[u] = i + u * 256 < n ? in[i + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
	for (int u = 0; u < U; u++) {
		size_t j = i + u * 256;
		if (j < n) {
			/* output piece pair of input piece j: 2 consecutive pieces of
			 * a 512-B (per 256 lanes x 16 B x 2) run */
			size_t blk = j / 256, l = j % 256;
			u32x4 *o = out + blk * 512;
			__builtin_nontemporal_store(v[u], o + l);
			__builtin_nontemporal_store(v[u] + 1u, o + 256 + l);
		}
	}
}

template <int U>
__global__ __launch_bounds__(256) void
k_copy(const u32x4 *__restrict__ in, u32x4 *__restrict__ out, size_t n)
{
	size_t i = ((size_t)blockIdx.x * 256 * U) + threadIdx.x;
	u32x4 v[U];
#pragma unroll
	for (int u = 0; u < U; u++)
		v[u] = i + u * 256 < n ? in[i + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
	for (int u = 0; u < U; u++)
		if (i + u * 256 < n)
			__builtin_nontemporal_store(v[u], out + i + u * 256);
}

template <int U>
__global__ __launch_bounds__(256) void
k_read(const u32x4 *__restrict__ in, uint32_t *sink, size_t n)
{
	size_t i = ((size_t)blockIdx.x * 256 * U) + threadIdx.x;
	uint32_t acc = 0;
#pragma unroll
	for (int u = 0; u < U; u++)
		if (i + u * 256 < n) {
			u32x4 v = in[i + u * 256];
			acc ^= v.x ^ v.y ^ v.z ^ v.w;
		}
	if (acc == 0x12345678u)
		*sink = acc;
}

template <int U>
__global__ __launch_bounds__(256) void
k_write(u32x4 *__restrict__ out, size_t n)
{
	size_t i = ((size_t)blockIdx.x * 256 * U) + threadIdx.x;
#pragma unroll
	for (int u = 0; u < U; u++)
		if (i + u * 256 < n)
			__builtin_nontemporal_store(u32x4{(uint32_t)i, 1, 2, 3},
			    out + i + u * 256);
}

template <typename F>
static float
timeit(F f)
{
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	f();
	f();
	hipDeviceSynchronize();
	hipEventRecord(a, 0);
	for (int i = 0; i < 20; i++)
		f();
	hipEventRecord(b, 0);
	hipEventSynchronize(b);
	float ms;
	hipEventElapsedTime(&ms, a, b);
	hipEventDestroy(a);
	hipEventDestroy(b);
	return ms / 20;
}

int
main()
{
	const size_t R = 330000000, n = R / 16;
	u32x4 *in, *out;
	uint32_t *sink;
	CHECK(hipMalloc(&in, R));
	CHECK(hipMalloc(&out, 2 * R + 8192));
	CHECK(hipMalloc(&sink, 4));
	CHECK(hipMemset(in, 1, R));
	const unsigned g4 = (unsigned)((n + 1023) / 1024), g1 = (unsigned)((n + 255) / 256);
	float t_exp4 = timeit([&] { k_expand<4><<<g4, 256>>>(in, out, n); });
	float t_exp1 = timeit([&] { k_expand<1><<<g1, 256>>>(in, out, n); });
	float t_cp4 = timeit([&] { k_copy<4><<<g4, 256>>>(in, out, n); });
	float t_rd4 = timeit([&] { k_read<4><<<g4, 256>>>(in, sink, n); });
	float t_wr4 = timeit([&] { k_write<4><<<(unsigned)((2 * n + 1023) / 1024), 256>>>(out, 2 * n); });
	CHECK(hipDeviceSynchronize());
	printf("{\"expand4_ms\": %.4f, \"expand4_TBs\": %.3f, \"expand1_TBs\": %.3f, "
	    "\"copy4_TBs\": %.3f, \"read4_TBs\": %.3f, \"write4_TBs\": %.3f}\n",
	    t_exp4, 3 * R / t_exp4 / 1e9, 3 * R / t_exp1 / 1e9, 2 * R / t_cp4 / 1e9,
	    R / t_rd4 / 1e9, 2 * R / t_wr4 / 1e9);
	return 0;
}
