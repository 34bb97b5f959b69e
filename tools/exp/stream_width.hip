// Element passes over lane-private int16 windows on gfx950, by access width.
// Each lane owns 16 windows of 328 int16 (10.5 KB, the lane analysis'
// working-set size, so the passes stream from beyond the caches as the
// codec's do); pass p rescales window p % 16 in place (y = x >> s, a
// stateful running sum added so each element depends on the previous):
//   mode 0: 2-byte loads / stores, eight loads issued ahead (dsp.h v_batch)
//   mode 1: 4-byte loads / stores (sample pairs)
//   mode 2: 16-byte loads / stores (eight samples), two chunks ahead
// 4,096 one-wave blocks (4 waves per SIMD, as k_enc_ana at 262,144 ch).
//   hipcc -O3 --offload-arch=gfx950 tools/exp/stream_width.hip -o build/exp/stream_width
#include <hip/hip_runtime.h>
#include <stdio.h>

#define W 328
#define NW 16
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int16_t f(int16_t x, int s, int &acc)
{
	acc += x;
	return (int16_t) ((x >> s) + (acc & 1));
}

template <int MODE>
__global__ __launch_bounds__(64, 4) void k(int *out, int passes, int s)
{
	__attribute__((aligned(16))) int16_t buf[NW][W];
	const int lane = threadIdx.x;
	for (int w = 0; w < NW; w++)
		for (int i = 0; i < W; i++)
			buf[w][i] = (int16_t) (i * 31 + w * 7 + lane);
	int acc = 0;
	for (int p = 0; p < passes; p++) {
		int16_t *x = buf[(p * 5 + s) & (NW - 1)];
		if (MODE == 0) {
			int16_t v[8];
			for (int q = 0; q < 8; q++)
				v[q] = x[q];
			int i = 0;
			for (; i + 16 <= W; i += 8) {
				int16_t nv[8];
				for (int q = 0; q < 8; q++)
					nv[q] = x[i + 8 + q];
				for (int q = 0; q < 8; q++)
					x[i + q] = f(v[q], s, acc);
				for (int q = 0; q < 8; q++)
					v[q] = nv[q];
			}
			for (int q = 0; q < 8; q++)
				x[i + q] = f(v[q], s, acc);
		} else if (MODE == 1) {
			uint32_t *d = (uint32_t *) x;
			uint32_t v[4];
			for (int q = 0; q < 4; q++)
				v[q] = d[q];
			int i = 0;
			for (; i + 8 <= W / 2; i += 4) {
				uint32_t nv[4];
				for (int q = 0; q < 4; q++)
					nv[q] = d[i + 4 + q];
				for (int q = 0; q < 4; q++) {
					uint32_t lo = (uint16_t) f((int16_t) v[q], s, acc);
					uint32_t hi = (uint16_t) f((int16_t) (v[q] >> 16), s, acc);
					d[i + q] = lo | hi << 16;
				}
				for (int q = 0; q < 4; q++)
					v[q] = nv[q];
			}
			for (int q = 0; q < 4; q++) {
				uint32_t lo = (uint16_t) f((int16_t) v[q], s, acc);
				uint32_t hi = (uint16_t) f((int16_t) (v[q] >> 16), s, acc);
				d[i + q] = lo | hi << 16;
			}
		} else {
			u4 *d = (u4 *) x;
			const int nc = W / 8;	/* 41 */
			u4 c0 = d[0], c1 = d[1];
			for (int c = 0; c < nc; c++) {
				u4 nx = d[c + 2 < nc ? c + 2 : nc - 1];
				u4 y;
				for (int q = 0; q < 4; q++) {
					uint32_t lo = (uint16_t) f((int16_t) c0[q], s, acc);
					uint32_t hi = (uint16_t) f((int16_t) (c0[q] >> 16), s, acc);
					y[q] = lo | hi << 16;
				}
				d[c] = y;
				c0 = c1;
				c1 = nx;
			}
		}
	}
	int r = acc;
	for (int w = 0; w < NW; w++)
		r += buf[w][(lane * 3 + w) % W];
	out[blockIdx.x * 64 + lane] = r;
}

int main()
{
	int *out;
	const int blocks = 4096, passes = 256;
	(void) hipMalloc(&out, sizeof(int) * blocks * 64);
	hipEvent_t a, b;
	(void) hipEventCreate(&a);
	(void) hipEventCreate(&b);
	void (*ks[])(int *, int, int) = {k<0>, k<1>, k<2>};
	for (int m = 0; m < 3; m++) {
		ks[m]<<<blocks, 64>>>(out, passes, 1);
		(void) hipEventRecord(a);
		ks[m]<<<blocks, 64>>>(out, passes, 2);
		(void) hipEventRecord(b);
		(void) hipEventSynchronize(b);
		float ms;
		(void) hipEventElapsedTime(&ms, a, b);
		printf("mode %d: %.3f ms, %.2f us per 328-sample pass (all waves)\n", m, ms, ms * 1e3 / passes);
	}
	return 0;
}
