// CPU check of orbmi::fast_arc_strength (csrc/fast_score.h) against a scalar restatement of
// FAST_t<16>'s segment test and cornerScore<16> (OpenCV 3.2 fast.cpp / fast_score.cpp, as used
// at src/ORBextractor.cc:809-816; the same restatement as oracle/orb_extract_oracle.cpp:205).
// For every patch and thresholds t >= th: passes(t) == (S > t), and for a pixel passing at th,
// cornerScore(th) == S - 1.  Built with hipcc as a host program by tests/test_fast_score.py.
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#include "../../orb_slam2_with_comment_amd/csrc/fast_score.h"

static bool segment(int v, const int p[16], int t) {
    for (int s = 0; s < 16; s++) {
        bool br = true, dk = true;
        for (int k = 0; k < 9; k++) {
            const int x = p[(s + k) & 15];
            br &= x > v + t;
            dk &= x < v - t;
        }
        if (br || dk) return true;
    }
    return false;
}

static int corner_score(int v, const int p[16], int th) {
    int d[25];
    for (int k = 0; k < 25; k++) d[k] = v - p[k & 15];
    int a0 = th;
    for (int k = 0; k < 16; k += 2) {
        int a = d[k + 1] < d[k + 2] ? d[k + 1] : d[k + 2];
        a = a < d[k + 3] ? a : d[k + 3];
        if (a <= a0) continue;
        for (int j = 4; j <= 8; j++) a = a < d[k + j] ? a : d[k + j];
        const int u = a < d[k] ? a : d[k], w = a < d[k + 9] ? a : d[k + 9];
        a0 = a0 > u ? a0 : u;
        a0 = a0 > w ? a0 : w;
    }
    int b0 = -a0;
    for (int k = 0; k < 16; k += 2) {
        int b = d[k + 1] > d[k + 2] ? d[k + 1] : d[k + 2];
        for (int j = 3; j <= 5; j++) b = b > d[k + j] ? b : d[k + j];
        if (b >= b0) continue;
        for (int j = 6; j <= 8; j++) b = b > d[k + j] ? b : d[k + j];
        const int u = b > d[k] ? b : d[k], w = b > d[k + 9] ? b : d[k + 9];
        b0 = b0 < u ? b0 : u;
        b0 = b0 < w ? b0 : w;
    }
    return (-b0 - 1) & 0xFF;
}

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static unsigned rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return (unsigned)(rs >> 11);
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    long bad = 0, corners = 0;
    for (long it = 0; it < n; it++) {
        int p[16], v;
        const int mode = it % 4;
        v = rnd() & 255;
        for (int k = 0; k < 16; k++) {
            if (mode == 0) p[k] = rnd() & 255;                                   // uniform
            else if (mode == 1) p[k] = v + (int)(rnd() % 81) - 40;               // near the centre
            else if (mode == 2) p[k] = (rnd() & 1) ? (rnd() & 255) : v;          // ties with the centre
            else p[k] = (k - (int)(it >> 2) % 16 + 16) % 16 < 10 ? v + 30 + (int)(rnd() % 20) : rnd() & 255;  // arcs
            p[k] = p[k] < 0 ? 0 : p[k] > 255 ? 255 : p[k];
        }
        const int th = rnd() % 40;
        const int S = orbmi::fast_arc_strength(v, p, th);
        for (int t = th; t < th + 60; t += 7)
            if (segment(v, p, t) != (S > t)) bad++;
        if (segment(v, p, th)) {
            corners++;
            if (corner_score(v, p, th) != S - 1) bad++;
        }
    }
    printf("patches %ld corners %ld mismatches %ld\n", n, corners, bad);
    return bad != 0;
}
