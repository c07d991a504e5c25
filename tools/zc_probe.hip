/*
 * zc_probe.hip -- kernel reads and writes of host memory over PCIe (VERDICT
 * r05 item 6: the duplex probe saw a kernel read pinned host memory at 22
 * GB/s and write it at 46).  Sweeps, one factor at a time:
 *   - the host memory: hipHostMalloc (coherent, the default), hipHostMalloc
 *     NonCoherent, and malloc'ed memory registered with hipHostRegister;
 *   - loads in flight per lane (U = 1, 4, 16 independent 16-B loads) and
 *     the grid (256 or 1024 workgroups of 256 threads);
 * against the copy engines (hipMemcpyAsync H2D / D2H of the same buffer).
 * Each case: median of 7 timed passes over a 256 MiB buffer (hipEvents).
 *
 * build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/zc_probe tools/zc_probe.hip
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
	fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
#define BYTES (256ull << 20)

template <int U>
__global__ __launch_bounds__(256) void
kread(const u32x4 *in, uint64_t n, u32x4 *sink)
{
	u32x4 acc = { 0u, 0u, 0u, 0u };
	const uint64_t step = (uint64_t)gridDim.x * 256u * U;
	for (uint64_t b = (uint64_t)blockIdx.x * 256u * U + threadIdx.x; b < n; b += step) {
		u32x4 v[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			v[u] = b + (uint64_t)u * 256u < n ? in[b + (uint64_t)u * 256u] :
			    (u32x4){ 0u, 0u, 0u, 0u };
#pragma unroll
		for (int u = 0; u < U; u++)
			acc ^= v[u];
	}
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u)
		sink[threadIdx.x] = acc;	/* practically never: keeps the loads */
}

__global__ __launch_bounds__(256) void
kwrite(u32x4 *out, uint64_t n)
{
	const u32x4 v = { threadIdx.x, blockIdx.x, 1u, 2u };
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n;
	    i += (uint64_t)gridDim.x * 256u)
		out[i] = v;
}

static u32x4 *g_sink;

/* read n16 pieces of host memory into HBM while writing m16 pieces of HBM
 * to host memory: both PCIe directions from one kernel */
__global__ __launch_bounds__(256) void
kduplex(const u32x4 *hin, u32x4 *dmid, uint64_t n16, const u32x4 *dsrc, u32x4 *hout,
    uint64_t m16)
{
	const uint64_t step = (uint64_t)gridDim.x * 256u;
	const uint64_t i0 = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	for (uint64_t i = i0; i < n16 || i < m16; i += step) {
		if (i < n16)
			dmid[i] = hin[i];
		if (i < m16)
			hout[i] = dsrc[i];
	}
}

template <typename F>
static double
timeit(F &&f)
{
	hipEvent_t a, b;
	CHECK(hipEventCreate(&a));
	CHECK(hipEventCreate(&b));
	std::vector<float> ms;
	for (int it = 0; it < 9; it++) {
		CHECK(hipEventRecord(a, 0));
		f();
		CHECK(hipEventRecord(b, 0));
		CHECK(hipEventSynchronize(b));
		float t;
		CHECK(hipEventElapsedTime(&t, a, b));
		if (it >= 2)
			ms.push_back(t);
	}
	std::sort(ms.begin(), ms.end());
	CHECK(hipEventDestroy(a));
	CHECK(hipEventDestroy(b));
	return ms[ms.size() / 2];
}

static void
report(const char *mem, const char *op, int grid, int u, double ms)
{
	printf("{\"memory\": \"%s\", \"op\": \"%s\", \"grid\": %d, \"loads_per_lane\": %d, "
	    "\"ms\": %.3f, \"GBps\": %.1f}\n", mem, op, grid, u, ms, BYTES / ms / 1e6);
	fflush(stdout);
}

static void
sweep(const char *mem, void *host_dev_ptr, void *host_ptr, void *dbuf)
{
	const uint64_t n = BYTES / 16;
	const u32x4 *in = (const u32x4 *)host_dev_ptr;
	for (int grid : { 256, 1024 }) {
		report(mem, "kernel read", grid, 1, timeit([&] {
			hipLaunchKernelGGL(kread<1>, dim3(grid), dim3(256), 0, 0, in, n, g_sink); }));
		report(mem, "kernel read", grid, 4, timeit([&] {
			hipLaunchKernelGGL(kread<4>, dim3(grid), dim3(256), 0, 0, in, n, g_sink); }));
		report(mem, "kernel read", grid, 16, timeit([&] {
			hipLaunchKernelGGL(kread<16>, dim3(grid), dim3(256), 0, 0, in, n, g_sink); }));
		report(mem, "kernel write", grid, 1, timeit([&] {
			hipLaunchKernelGGL(kwrite, dim3(grid), dim3(256), 0, 0,
			    (u32x4 *)host_dev_ptr, n); }));
	}
	report(mem, "copy engine H2D", 0, 0, timeit([&] {
		CHECK(hipMemcpyAsync(dbuf, host_ptr, BYTES, hipMemcpyHostToDevice, 0)); }));
	report(mem, "copy engine D2H", 0, 0, timeit([&] {
		CHECK(hipMemcpyAsync(host_ptr, dbuf, BYTES, hipMemcpyDeviceToHost, 0)); }));
}

/* both directions at once: kernel-initiated, and kernel beside the copy
 * engine (XA-sized reads of 132 MB against PCM-sized writes of 256 MB, the
 * 2M-eblock stereo call's shape) */
static void
duplex(void *dp_in, void *h_in, void *dp_out, void *h_out, void *dbuf, void *dbuf2)
{
	const uint64_t nin = 132000000ull / 16, nout = 256000000ull / 16;
	hipStream_t s2;
	CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
	const double t_one = timeit([&] {
		hipLaunchKernelGGL(kduplex, dim3(1024), dim3(256), 0, 0, (const u32x4 *)dp_in,
		    (u32x4 *)dbuf, nin, (const u32x4 *)dbuf2, (u32x4 *)dp_out, nout); });
	printf("{\"duplex\": \"one kernel: 132 MB host->HBM reads + 256 MB HBM->host writes\", "
	    "\"ms\": %.3f, \"GBps_total\": %.1f}\n", t_one, 388e6 / t_one / 1e6);
	hipEvent_t e0, e1;
	CHECK(hipEventCreate(&e0));
	CHECK(hipEventCreate(&e1));
	const double t_kr_dma = timeit([&] {
		CHECK(hipEventRecord(e0, 0));
		CHECK(hipStreamWaitEvent(s2, e0, 0));
		CHECK(hipMemcpyAsync(h_out, dbuf2, 256000000ull, hipMemcpyDeviceToHost, s2));
		hipLaunchKernelGGL(kduplex, dim3(1024), dim3(256), 0, 0, (const u32x4 *)dp_in,
		    (u32x4 *)dbuf, nin, (const u32x4 *)dbuf2, (u32x4 *)dp_out, (uint64_t)0);
		CHECK(hipEventRecord(e1, s2));
		CHECK(hipStreamWaitEvent(0, e1, 0)); });
	printf("{\"duplex\": \"kernel reads 132 MB host->HBM beside copy-engine D2H of 256 MB\", "
	    "\"ms\": %.3f, \"GBps_total\": %.1f}\n", t_kr_dma, 388e6 / t_kr_dma / 1e6);
	const double t_kw_dma = timeit([&] {
		CHECK(hipEventRecord(e0, 0));
		CHECK(hipStreamWaitEvent(s2, e0, 0));
		CHECK(hipMemcpyAsync(dbuf, h_in, 132000000ull, hipMemcpyHostToDevice, s2));
		hipLaunchKernelGGL(kduplex, dim3(1024), dim3(256), 0, 0, (const u32x4 *)dp_in,
		    (u32x4 *)dbuf, (uint64_t)0, (const u32x4 *)dbuf2, (u32x4 *)dp_out, nout);
		CHECK(hipEventRecord(e1, s2));
		CHECK(hipStreamWaitEvent(0, e1, 0)); });
	printf("{\"duplex\": \"kernel writes 256 MB HBM->host beside copy-engine H2D of 132 MB\", "
	    "\"ms\": %.3f, \"GBps_total\": %.1f}\n", t_kw_dma, 388e6 / t_kw_dma / 1e6);
	fflush(stdout);
	CHECK(hipStreamDestroy(s2));
}

int
main()
{
	void *dbuf, *h, *dp;
	CHECK(hipMalloc(&dbuf, BYTES));
	CHECK(hipMalloc(&g_sink, 256 * 16));
	/* device-memory reference for the same kernels */
	report("device HBM", "kernel read", 1024, 4, timeit([&] {
		hipLaunchKernelGGL(kread<4>, dim3(1024), dim3(256), 0, 0, (const u32x4 *)dbuf,
		    BYTES / 16, g_sink); }));

	CHECK(hipHostMalloc(&h, BYTES, hipHostMallocDefault));
	memset(h, 1, BYTES);
	CHECK(hipHostGetDevicePointer(&dp, h, 0));
	sweep("hipHostMalloc (coherent)", dp, h, dbuf);
	CHECK(hipHostFree(h));

	CHECK(hipHostMalloc(&h, BYTES, hipHostMallocNonCoherent));
	memset(h, 1, BYTES);
	CHECK(hipHostGetDevicePointer(&dp, h, 0));
	sweep("hipHostMalloc NonCoherent", dp, h, dbuf);
	CHECK(hipHostFree(h));

	{
		void *hi, *ho, *di, *dout, *dbuf2;
		CHECK(hipHostMalloc(&hi, BYTES, hipHostMallocDefault));
		CHECK(hipHostMalloc(&ho, BYTES, hipHostMallocDefault));
		memset(hi, 1, BYTES);
		memset(ho, 2, BYTES);
		CHECK(hipHostGetDevicePointer(&di, hi, 0));
		CHECK(hipHostGetDevicePointer(&dout, ho, 0));
		CHECK(hipMalloc(&dbuf2, BYTES));
		duplex(di, hi, dout, ho, dbuf, dbuf2);
		CHECK(hipHostFree(hi));
		CHECK(hipHostFree(ho));
		CHECK(hipFree(dbuf2));
	}
	{	/* registration cost of pageable buffers of the call's sizes */
		for (size_t sz : { (size_t)132000000, (size_t)256000000 }) {
			void *p = aligned_alloc(4096, (sz + 4095) / 4096 * 4096);
			memset(p, 3, sz);
			std::vector<double> ts;
			for (int k = 0; k < 5; k++) {
				hipEvent_t a;
				CHECK(hipEventCreate(&a));
				const auto t0 = std::chrono::steady_clock::now();
				CHECK(hipHostRegister(p, sz, hipHostRegisterMapped));
				const auto t1 = std::chrono::steady_clock::now();
				CHECK(hipHostUnregister(p));
				ts.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
				CHECK(hipEventDestroy(a));
			}
			std::sort(ts.begin(), ts.end());
			printf("{\"register_bytes\": %zu, \"ms_median\": %.3f}\n", sz, ts[2]);
			free(p);
		}
	}
	h = aligned_alloc(4096, BYTES);
	memset(h, 1, BYTES);
	CHECK(hipHostRegister(h, BYTES, hipHostRegisterMapped));
	CHECK(hipHostGetDevicePointer(&dp, h, 0));
	sweep("malloc + hipHostRegister", dp, h, dbuf);
	CHECK(hipHostUnregister(h));
	free(h);
	return 0;
}
