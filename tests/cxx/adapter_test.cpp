// Drives the C++ adapter (orc_amd/csrc/GpuRleDecoder.hh) the way the
// reference's gtest helpers drive orc::RleDecoder (c++/test/TestRleDecoder.cc:
// 30-56: read with batch sizes 1, 3, 7 and all at once, compare non-null
// slots). Input: lines "<kind> <signed> <hex> <n> <v0> ... " where kind is
// rlev2 | byte | bool and a value "x" means "not asserted".
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../orc_amd/csrc/GpuRleDecoder.hh"

using namespace orcg::cxx;

static std::vector<uint8_t> unhex(const std::string& h) {
  std::vector<uint8_t> b(h.size() / 2);
  for (size_t i = 0; i < b.size(); ++i) b[i] = (uint8_t)std::stoi(h.substr(2 * i, 2), nullptr, 16);
  return b;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::ifstream in(argv[1]);
  Context ctx(0);
  std::string line;
  int cases = 0, failures = 0;
  while (std::getline(in, line)) {
    std::istringstream ss(line);
    std::string kind, hex;
    int sgn;
    size_t n;
    ss >> kind >> sgn >> hex >> n;
    std::vector<std::string> exp(n);
    for (auto& e : exp) ss >> e;
    const std::vector<uint8_t> data = unhex(hex);
    for (size_t batch : {size_t(1), size_t(3), size_t(7), n}) {
      std::vector<int64_t> got;
      if (kind == "rlev2") {
        auto rle = createGpuRleDecoder(ctx, data.data(), data.size(), sgn != 0);
        for (size_t i = 0; i < n; i += batch) {
          std::vector<int64_t> d(std::min(batch, n - i));
          rle->next(d.data(), d.size(), nullptr);
          got.insert(got.end(), d.begin(), d.end());
        }
      } else {
        auto rle = kind == "bool" ? createGpuBooleanRleDecoder(ctx, data.data(), data.size())
                                  : createGpuByteRleDecoder(ctx, data.data(), data.size());
        for (size_t i = 0; i < n; i += batch) {
          std::vector<char> d(std::min(batch, n - i));
          rle->next(d.data(), d.size(), nullptr);
          for (char c : d) got.push_back((uint8_t)c);
        }
      }
      for (size_t i = 0; i < n; ++i) {
        if (exp[i] == "x") continue;
        if (std::stoll(exp[i]) != got[i]) {
          std::cerr << "mismatch line " << cases << " batch " << batch << " at " << i << ": " << exp[i]
                    << " vs " << got[i] << "\n";
          ++failures;
          break;
        }
      }
    }
    ++cases;
  }
  // ParseError surfaces as the reference's exception type and message
  {
    const uint8_t bad[] = {0x8E, 0x09, 0x2B, 0x20, 0x07, 0xD0};
    auto rle = createGpuRleDecoder(ctx, bad, sizeof bad, false);
    int64_t v[10];
    try {
      rle->next(v, 10, nullptr);
      std::cerr << "no ParseError for pl==0\n";
      ++failures;
    } catch (const ParseError& e) {
      if (std::string(e.what()) != "Corrupt PATCHED_BASE encoded data (pl==0)!") {
        std::cerr << "pl==0 message: " << e.what() << "\n";
        ++failures;
      }
    } catch (const std::exception& e) {
      std::cerr << "pl==0 wrong exception type: " << e.what() << "\n";
      ++failures;
    }
  }
  // seek through a PositionProvider (c++/test/TestRleDecoder.cc:717-744)
  {
    const uint8_t bytes[] = {0x42, 0x13, 0x22, 0x22, 0x22, 0x22, 0x22, 0x46, 0x13, 0x04,
                             0x04, 0x04, 0x04, 0x04, 0x04, 0x04, 0x04, 0x04, 0x04};
    auto rle = createGpuRleDecoder(ctx, bytes, sizeof bytes, true);
    PositionProvider loc({7, 13});
    rle->seek(loc);
    int64_t d[3];
    rle->next(d, 3, nullptr);
    if (d[0] != 2 || d[1] != 0 || d[2] != 2) {
      std::cerr << "seek: " << d[0] << " " << d[1] << " " << d[2] << "\n";
      ++failures;
    }
  }
  std::printf("%s %d cases, %d failures\n", failures ? "FAIL" : "OK", cases, failures);
  return failures ? 1 : 0;
}
