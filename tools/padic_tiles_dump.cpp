// Writes the fthe_padic_m37 LDS tile image of P (hex argv[1]) to argv[2]: the host builder
// (fedtree_amd/csrc/padic_tiles.hpp) checked byte for byte against tools/padic_mfma_model.py.
#include "../fedtree_amd/csrc/padic_tiles.hpp"
#include <cstdio>
int main(int argc, char **argv) {
    if (argc != 3) return 2;
    mpz_t P;
    mpz_init_set_str(P, argv[1], 16);
    std::vector<uint8_t> img = padic_tiles::build(P);
    if (img.empty()) return 1;
    FILE *f = fopen(argv[2], "wb");
    if (!f) return 3;
    fwrite(img.data(), 1, img.size(), f);
    fclose(f);
    return 0;
}
