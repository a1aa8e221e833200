// C++ drop-in check (include/orbmi.hpp): a Frame-constructor-shaped call sequence on a raw u8
// stereo pair.  Usage: dropin_extract LEFT.raw RIGHT.raw rows cols bf fx OUT.bin
// OUT.bin = int32 n, n x orbmi_keypoint, n x 32 descriptor bytes, n x float u_right, n x float depth,
// then the scale factors (int32 nlevels + floats).  tests/test_cpp_dropin.py compares it with
// the oracle.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <thread>

#include "orbmi.hpp"

static std::vector<uint8_t> read_raw(const char* path, size_t n) {
    std::vector<uint8_t> v(n);
    std::ifstream f(path, std::ios::binary);
    if (!f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)n)) throw std::runtime_error("short read");
    return v;
}

int main(int argc, char** argv) {
    if (argc != 8) {
        std::cerr << "usage: dropin_extract LEFT.raw RIGHT.raw rows cols bf fx OUT.bin\n";
        return 2;
    }
    const int rows = std::atoi(argv[3]), cols = std::atoi(argv[4]);
    const float bf = std::strtof(argv[5], nullptr), fx = std::strtof(argv[6], nullptr);
    try {
        const auto L = read_raw(argv[1], (size_t)rows * cols), R = read_raw(argv[2], (size_t)rows * cols);
        // Tracking::Tracking constructs one extractor per camera (src/Tracking.cc:120-126)
        orbmi::ORBextractor left(2000, 1.2f, 8, 20, 7), right(2000, 1.2f, 8, 20, 7);
        std::vector<orbmi::KeyPoint> kl, kr;
        std::vector<uint8_t> dl, dr;
        // Frame::Frame runs both extractions on two threads (src/Frame.cc:78-81)
        std::thread tl([&] { left(L.data(), rows, cols, cols, kl, dl); });
        std::thread tr([&] { right(R.data(), rows, cols, cols, kr, dr); });
        tl.join();
        tr.join();
        std::vector<float> uR, depth;
        orbmi::ComputeStereoMatches(left, right, bf, fx, (int)kl.size(), uR, depth);
        std::ofstream o(argv[7], std::ios::binary);
        const int n = (int)kl.size();
        o.write(reinterpret_cast<const char*>(&n), 4);
        o.write(reinterpret_cast<const char*>(kl.data()), (std::streamsize)(n * sizeof(orbmi::KeyPoint)));
        o.write(reinterpret_cast<const char*>(dl.data()), (std::streamsize)dl.size());
        o.write(reinterpret_cast<const char*>(uR.data()), (std::streamsize)(n * 4));
        o.write(reinterpret_cast<const char*>(depth.data()), (std::streamsize)(n * 4));
        const auto sf = left.GetScaleFactors();
        const int nl = (int)sf.size();
        o.write(reinterpret_cast<const char*>(&nl), 4);
        o.write(reinterpret_cast<const char*>(sf.data()), nl * 4);
        std::cout << "keypoints " << n << " right " << kr.size() << "\n";
    } catch (const std::exception& e) {
        std::cerr << "error: " << e.what() << "\n";
        return 1;
    }
    return 0;
}
