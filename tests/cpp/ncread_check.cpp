// CPU check of include/harp_amd/ncread.hpp: prints every requested variable of
// a classic or netCDF-4 file as "name i value" lines (tests/test_ncread.py,
// tests/test_nc4read.py); a leading "--classic" forces the classic reader.
#include <harp_amd/ncread.hpp>

#include <cstdio>

int main(int argc, char** argv) {
  try {
    const bool classic = argc > 1 && std::string(argv[1]) == "--classic";
    if (classic) {
      ++argv;
      --argc;
    }
    std::unique_ptr<harp_amd::NetCDFClassic> cl;
    std::unique_ptr<harp_amd::NetCDFFile> any;
    if (classic)
      cl = std::make_unique<harp_amd::NetCDFClassic>(argv[1]);
    else
      any = std::make_unique<harp_amd::NetCDFFile>(argv[1]);
    auto dim_len = [&](std::string const& n) { return cl ? cl->dim_len(n) : any->dim_len(n); };
    auto var = [&](std::string const& n) { return cl ? cl->var(n) : any->var(n); };
    for (int a = 2; a < argc; ++a) {
      std::string name = argv[a];
      if (name.rfind("dim:", 0) == 0) {
        std::printf("%s %zu\n", name.c_str(), dim_len(name.substr(4)));
        continue;
      }
      auto v = var(name);
      for (size_t i = 0; i < v.size(); ++i) std::printf("%s %zu %.17g\n", name.c_str(), i, v[i]);
    }
  } catch (std::exception const& e) {
    std::printf("error %s\n", e.what());
    return 2;
  }
  return 0;
}
