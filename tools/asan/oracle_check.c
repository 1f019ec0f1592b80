/* Host AddressSanitizer / UBSan check of the CPU oracle (test infrastructure): every
 * oracle entry point on small, exactly-sized heap buffers, incl. taps far outside the
 * image, NaN / infinite coordinates and degenerate 1-pixel frames. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../oracle/mpiv_oracle.h"

static float *buf(size_t n, float v) {
    float *p = (float *)malloc(n * sizeof(float));
    for (size_t i = 0; i < n; ++i) p[i] = v + 0.001f * (float)(i % 97);
    return p;
}

int main(void) {
    const int B = 2, H = 5, W = 7, P = 3;
    const int64_t st5[5] = {(int64_t)H * W * P * 4, W * P * 4, P * 4, 4, 1};
    float *mpi = buf((size_t)B * H * W * P * 4, 0.2f);
    float *homs = buf((size_t)B * P * 9, 0.0f);
    for (int k = 0; k < B * P; ++k) {  /* identity-ish, one with w == 0 and one with huge shifts */
        float *h = homs + k * 9;
        h[0] = 1.0f; h[4] = 1.0f; h[8] = k == 1 ? 0.0f : 1.0f; h[2] = k == 2 ? 1e30f : 0.3f;
    }
    float *out = buf((size_t)B * H * W * 4, 0.0f);
    oracle_render(mpi, st5, B, H, W, P, homs, out, 2);
    oracle_render_ct(mpi, st5, B, H, W, P, 1, 3, 0, homs, out, 2);
    float *dout = buf((size_t)B * H * W * 3, 0.5f), *dmpi = buf((size_t)B * H * W * P * 4, 0.0f);
    oracle_render_backward(mpi, st5, B, H, W, P, homs, dout, dmpi, 8, 2);
    const int64_t st4[4] = {(int64_t)H * W * 3, W * 3, 3, 1};
    float *img = buf((size_t)B * H * W * 3, 0.1f), *ki = buf((size_t)B * 9, 0.01f), *proj = buf((size_t)B * 16, 0.2f);
    float depths[2] = {10.0f, NAN};
    float *psv = buf((size_t)B * H * W * 2 * 3, 0.0f);
    oracle_plane_sweep(img, st4, B, H, W, 3, ki, proj, depths, 2, H, W, psv, 2);
    float *dm = buf((size_t)B * H * W, 1.0f);
    oracle_inverse_warp(img, st4, B, H, W, 3, ki, proj, dm, H, W, psv, 2);
    float *syn = buf((size_t)H * W * P * 4, 0.0f);
    oracle_synth_mpi(3u, H, W, 0, P, syn);
    oracle_render_synth(3u, H, W, P, 0, P, 1, 0, homs, 1, 4, out, 2);
    oracle_render_synth(3u, 1, 1, P, 0, P, 1, 1, homs, 0, 1, out, 1);  /* 1x1 frame: divides by 0 */
    float layers[2 * 3 * 4];
    for (int i = 0; i < 24; ++i) layers[i] = 0.1f * i;
    float oc[3 * 3];
    oracle_over_composite(layers, 2, 3, oc);
    printf("oracle_check: ok\n");
    free(mpi); free(homs); free(out); free(dout); free(dmpi); free(img); free(ki); free(proj); free(psv); free(dm);
    free(syn);
    return 0;
}
