/* CPU restatement of numpy's legacy `np.random.seed(s); np.random.randint(0, n, B)`.
 *
 * TEST INFRASTRUCTURE ONLY (the checker for the device index generator; never
 * linked into the product).
 *
 * Call site being restated: /root/reference/replay_buffer.py:107
 *   indices = np.random.randint(0, self._size, batch_size)
 * Third-party algorithm (numpy is an unpinned dependency, requirements.txt:3,
 * ">=1.18.1"; verified here against numpy 2.2.6): the legacy RandomState is a
 * raw MT19937 (Matsumoto & Nishimura 1998, init_genrand seeding for an integer
 * seed); randint(0, n) with rng = n-1 draws `v = next_uint32() & mask` (mask =
 * smallest 2^k-1 >= rng) until v <= rng ("masked rejection", numpy
 * random/src/distributions: buffered_bounded_masked_uint32), and returns 0
 * without consuming a draw when rng == 0.
 * Pinned by tests/golden/randint.npz (generated with numpy itself).
 */
#include <stdint.h>

#define MT_N 624
#define MT_M 397

typedef struct { uint32_t mt[MT_N]; int pos; } oracle_mt_state;

void oracle_mt_seed(oracle_mt_state *s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < MT_N; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->pos = MT_N;
}

static void mt_twist(oracle_mt_state *s) {
    for (int i = 0; i < MT_N; i++) {
        uint32_t y = (s->mt[i] & 0x80000000u) | (s->mt[(i + 1) % MT_N] & 0x7fffffffu);
        uint32_t v = s->mt[(i + MT_M) % MT_N] ^ (y >> 1);
        if (y & 1u) v ^= 0x9908b0dfu;
        s->mt[i] = v;
    }
    s->pos = 0;
}

uint32_t oracle_mt_next(oracle_mt_state *s) {
    if (s->pos >= MT_N) mt_twist(s);
    uint32_t y = s->mt[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* randint(0, n, B) for 1 <= n <= 2^32; writes B int64 indices. */
void oracle_randint(oracle_mt_state *s, uint64_t n, int64_t B, int64_t *out) {
    uint64_t rng = n - 1;
    if (rng == 0) { for (int64_t i = 0; i < B; i++) out[i] = 0; return; }
    uint32_t mask = (uint32_t)rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    for (int64_t i = 0; i < B; i++) {
        uint32_t v;
        if (rng == 0xffffffffu) { v = oracle_mt_next(s); }
        else { do { v = oracle_mt_next(s) & mask; } while (v > (uint32_t)rng); }
        out[i] = (int64_t)v;
    }
}

int oracle_mt_state_bytes(void) { return (int)sizeof(oracle_mt_state); }
