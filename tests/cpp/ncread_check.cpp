// CPU check of include/harp_amd/ncread.hpp: prints every requested variable of
// a classic netCDF file as "name i value" lines (tests/test_ncread.py).
#include <harp_amd/ncread.hpp>

#include <cstdio>

int main(int argc, char** argv) {
  try {
    harp_amd::NetCDFClassic nc(argv[1]);
    for (int a = 2; a < argc; ++a) {
      std::string name = argv[a];
      if (name.rfind("dim:", 0) == 0) {
        std::printf("%s %zu\n", name.c_str(), nc.dim_len(name.substr(4)));
        continue;
      }
      auto v = nc.var(name);
      for (size_t i = 0; i < v.size(); ++i) std::printf("%s %zu %.17g\n", name.c_str(), i, v[i]);
    }
  } catch (std::exception const& e) {
    std::printf("error %s\n", e.what());
    return 2;
  }
  return 0;
}
