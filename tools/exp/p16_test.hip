// Experiment: P16 / v_map on private arrays at every alignment, on the
// device, against the plain loops (dsp.h).  Prints the failing cases.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "dsp.h"
using namespace mlp;

__global__ void k(int *out, int sel)
{
	int16_t a[80], b[80];
	int bad = 0, cs = 0;
	for (int o1 = 0; o1 < 4; o1++)
		for (int o2 = 0; o2 < 4; o2++)
			for (int n = 0; n < 14; n++) {
				for (int i = 0; i < 80; i++) {
					a[i] = (int16_t) (i * 977 + threadIdx.x * 13 + 5);
					b[i] = (int16_t) (-i * 31);
				}
				int16_t *d = b + 8 + o2;
				const int16_t *s = a + 8 + o1;
				int16_t exp[20];
				for (int i = 0; i < n; i++)
					exp[i] = sel == 0 ? s[i] : (sel == 1 ? shr(s[i], 2) : mult(d[i], 12345));
				if (sel == 0)
					v_copy(d, s, n);
				else if (sel == 1)
					v_equ_shr(d, s, 2, n);
				else
					v_scale(d, 12345, n);
				for (int i = 0; i < n; i++)
					if (d[i] != exp[i]) {
						bad++;
						cs = o1 * 1000 + o2 * 100 + n;
					}
				if (d[-1] != (int16_t) (-(7 + o2) * 31) || d[n] != (int16_t) (-(8 + o2 + n) * 31)) {
					bad += 1000;
					cs = o1 * 1000 + o2 * 100 + n;
				}
				Word32 r1 = L_v_inner(s, d, n, 0, 0, 1), r2 = 0;
				for (int i = 0; i < n; i++)
					r2 = L_mac(r2, s[i], d[i]);
				if (r1 != r2) {
					bad += 100000;
					cs = o1 * 1000 + o2 * 100 + n;
				}
			}
	out[2 * threadIdx.x] = bad;
	out[2 * threadIdx.x + 1] = cs;
}
int main()
{
	int *d;
	hipMalloc(&d, 128 * 4);
	for (int sel = 0; sel < 3; sel++) {
		k<<<1, 64>>>(d, sel);
		hipError_t e = hipDeviceSynchronize();
		int h[128];
		hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
		printf("sel %d: %s lane0 bad=%d case=%d lane5 bad=%d case=%d\n", sel, hipGetErrorString(e), h[0], h[1], h[10], h[11]);
	}
	return 0;
}
