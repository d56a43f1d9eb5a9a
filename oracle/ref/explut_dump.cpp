// explut_dump.cpp -- test infrastructure (oracle/_ref): compiles the reference's own header-only ExpLUT
// generator UNCHANGED from /root/reference (RayTracingInVulkan/src/Utilities/ExpLUT.hpp:10-24, included
// through -I, never copied) and writes the table the reference uploads (Scene.cpp:47: generateExpLUT(256, 0,
// 8)) as 256 x {float k, float b} little-endian to the file named by argv[1]. Built by `make -C oracle ref`.
#include <cstdio>

#include "RayTracingInVulkan/src/Utilities/ExpLUT.hpp"

int main(int argc, char** argv) {
    if (argc != 2) return 2;
    const std::vector<LinearSegment> t = generateExpLUT(256, 0, 8);
    FILE* f = std::fopen(argv[1], "wb");
    if (!f) return 1;
    const size_t n = std::fwrite(t.data(), sizeof(LinearSegment), t.size(), f);
    std::fclose(f);
    return n == 256 ? 0 : 1;
}
