/*
 * ORACLE (test infrastructure only) -- plain-C restatement of the Cython monotonic-alignment DP.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this (via ctypes,
 * as the checker). The product path is grad-tts_amd/csrc/mas.hip.
 *
 * Follows /root/reference/model/monotonic_align/core.pyx:
 *   maximum_path_each  core.pyx:9-35   (generated C: core.c:2653-2940)
 *   maximum_path_c     core.pyx:38-45  (prange over the batch; OpenMP is not enabled by
 *                                       setup.py:7-11, so the loop is serial there and here)
 * Bit-exactness details copied from the generated C (core.c:2848-2859):
 *   max(v_cur, v_prev) lowers to  (v_prev > v_cur) ? v_prev : v_cur
 *   the backtrack compare is a strict  value[i, y-1] < value[i-1, y-1]   (core.c:2907)
 * Pinned against the reference itself: tests/test_oracle_golden.py compares this against the
 * Cython module built from the reference sources (oracle/_ref) and the committed golden paths.
 */
#include <stdint.h>

static void maximum_path_each(int32_t *path, float *value, int64_t ty_max, int t_x, int t_y, float max_neg_val)
{
    int index = t_x - 1;
    for (int y = 0; y < t_y; ++y) {
        int lo = t_x + y - t_y; if (lo < 0) lo = 0;
        int hi = y + 1; if (hi > t_x) hi = t_x;
        for (int x = lo; x < hi; ++x) {
            float v_cur = (x == y) ? max_neg_val : value[(int64_t)x * ty_max + (y - 1)];
            float v_prev;
            if (x == 0) v_prev = (y == 0) ? 0.0f : max_neg_val;
            else        v_prev = value[(int64_t)(x - 1) * ty_max + (y - 1)];
            float m = (v_prev > v_cur) ? v_prev : v_cur;
            value[(int64_t)x * ty_max + y] = m + value[(int64_t)x * ty_max + y];
        }
    }
    for (int y = t_y - 1; y > -1; --y) {
        path[(int64_t)index * ty_max + y] = 1;
        if (index != 0 && (index == y ||
                           value[(int64_t)index * ty_max + (y - 1)] < value[(int64_t)(index - 1) * ty_max + (y - 1)]))
            index = index - 1;
    }
}

/* paths: int32[b, tx_max, ty_max] (must be zero on entry, as np.zeros in __init__.py:17);
 * values: float32[b, tx_max, ty_max], mutated in place exactly as maximum_path_c does. */
void oracle_maximum_path(int32_t *paths, float *values, const int32_t *t_xs, const int32_t *t_ys,
                         int64_t b, int64_t tx_max, int64_t ty_max, float max_neg_val)
{
    for (int64_t i = 0; i < b; ++i)
        maximum_path_each(paths + i * tx_max * ty_max, values + i * tx_max * ty_max, ty_max,
                          t_xs[i], t_ys[i], max_neg_val);
}
