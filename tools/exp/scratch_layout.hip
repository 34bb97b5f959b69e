// Private-segment (scratch) access cost on gfx950, by access pattern.
// Each lane owns a private int32 array a[N] (dynamic indices keep it in
// scratch); the kernels read it with
//   mode 0: uniform index (all lanes the same i), dword loads
//   mode 1: per-lane index (i + 37 * lane) mod N, dword loads
//   mode 2: per-lane index, but lanes in 8 groups of 8 with equal index
//   mode 3: uniform index, 16-byte loads (int4)
//   mode 4: per-lane index, 16-byte loads
// Run under rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum
// SQ_INSTS_VMEM_RD: cache accesses per load instruction tell whether the
// segment is interleaved per dword across the wave (uniform = 4 x 64 B) or
// laid out lane by lane (uniform = 64 lines).
//   hipcc -O3 --offload-arch=gfx950 tools/exp/scratch_layout.hip -o /tmp/sl
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N 1024

template <int MODE>
__global__ __launch_bounds__(64) void k(int *out, int iters, int seed)
{
	int a[N];
	const int lane = threadIdx.x;
	for (int i = 0; i < N; i++)
		a[(i * 7 + seed) & (N - 1)] = i ^ lane;
	int s = 0;
	for (int it = 0; it < iters; it++) {
		int base = (it * 61 + seed) & (N - 1);
		int idx;
		if (MODE == 0 || MODE == 3)
			idx = base;
		else if (MODE == 2)
			idx = (base + 37 * (lane >> 3)) & (N - 1);
		else
			idx = (base + 37 * lane) & (N - 1);
		if (MODE >= 3) {
			idx &= ~3;
			int4 v = *(int4 *) &a[idx];
			s += v.x ^ v.y ^ v.z ^ v.w;
		} else {
			s += a[idx];
		}
	}
	out[blockIdx.x * 64 + lane] = s;
}

int main()
{
	int *out;
	const int blocks = 4096, iters = 4096;
	hipMalloc(&out, sizeof(int) * blocks * 64);
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	void (*ks[])(int *, int, int) = {k<0>, k<1>, k<2>, k<3>, k<4>};
	for (int m = 0; m < 5; m++) {
		ks[m]<<<blocks, 64>>>(out, iters, 3);
		hipEventRecord(a);
		ks[m]<<<blocks, 64>>>(out, iters, 5);
		hipEventRecord(b);
		hipEventSynchronize(b);
		float ms;
		hipEventElapsedTime(&ms, a, b);
		printf("mode %d: %.3f ms, %.2f ns per load per wave\n", m, ms,
		       ms * 1e6 / ((double) iters * blocks / 1024));
	}
	return 0;
}
