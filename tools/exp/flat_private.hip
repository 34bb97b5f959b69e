// Experiment: does a __noinline__ device function work on a pointer to the
// caller's private (stack) array on gfx950?  Mode 0: global buffer; mode 1:
// private buffer; mode 2: private buffer + negative indexing.
#include <hip/hip_runtime.h>
#include <stdio.h>
__device__ __noinline__ int work(short *p, int n, int neg)
{
	int s = 0;
	for (int i = 0; i < n; i++)
		p[i] = (short) (i * 3 + threadIdx.x);
	short *q = p + n / 2;
	for (int i = -(neg ? n / 2 : 0); i < n / 2; i++)
		s += q[i];
	return s;
}
__global__ void k(int *out, short *gbuf, int mode)
{
	short loc[300];
	short *p = mode == 0 ? gbuf + 300 * threadIdx.x : loc;
	out[threadIdx.x] = work(p, 300, mode == 2);
}
int main(int argc, char **argv)
{
	int mode = atoi(argv[1]);
	int *d;
	short *g;
	hipMalloc(&d, 64 * 4);
	hipMalloc(&g, 64 * 300 * 2);
	k<<<1, 64>>>(d, g, mode);
	hipError_t e = hipDeviceSynchronize();
	int h[64];
	hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
	printf("mode %d: %s sum[0]=%d sum[5]=%d\n", mode, hipGetErrorString(e), h[0], h[5]);
	return e != hipSuccess;
}
