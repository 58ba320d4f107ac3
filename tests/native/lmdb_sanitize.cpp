// Host-side sanitizer driver for the native LMDB reader / writer (csrc/lmdb_io.cpp).
//
// Built by tests/test_native_sanitize_cpu.py with
//   g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=all
// and IAMD_LMDB_NO_PYTHON (no pybind11), then run:
//   1. round trip: environments of small inline values, values spilling into overflow pages
//      and enough keys for multi-level branch trees are written and every key read back
//      (get + ordered key walk), plus absent-key lookups;
//   2. fuzz: thousands of copies of a valid file with random byte flips and truncations are
//      opened and fully read — every outcome must be a value or a std::runtime_error, never
//      a read outside the mapping (ASan) or undefined behaviour (UBSan).
// Exit status 0 = clean; the sanitizers abort with a report otherwise.
#define IAMD_LMDB_NO_PYTHON 1
#include "../../imaginaire_amd/csrc/lmdb_io.cpp"

#include <cstdio>
#include <map>
#include <random>

using iamd::lmdb::Reader;

static std::string rand_bytes(std::mt19937_64& rng, size_t n) {
  std::string s(n, '\0');
  for (auto& c : s) c = static_cast<char>(rng() & 0xff);
  return s;
}

static int round_trip(const std::string& dir, std::mt19937_64& rng, size_t nkeys,
                      size_t max_val, uint32_t psize) {
  std::map<std::string, std::string> ref;
  while (ref.size() < nkeys) {
    char key[64];
    std::snprintf(key, sizeof(key), "seq_%06zu/frame_%04u", ref.size(),
                  static_cast<unsigned>(rng() % 10000));
    ref[key] = rand_bytes(rng, rng() % (max_val + 1));
  }
  std::vector<std::pair<std::string, std::string>> kv(ref.begin(), ref.end());
  iamd::lmdb::write_lmdb(dir, kv, psize);
  Reader r(dir);
  if (r.entries() != ref.size()) return std::fprintf(stderr, "entries mismatch\n"), 1;
  for (const auto& it : ref) {
    auto v = r.get(it.first);
    if (!v.first || std::string(v.first, v.second) != it.second)
      return std::fprintf(stderr, "value mismatch for %s\n", it.first.c_str()), 1;
  }
  auto keys = r.keys();
  if (keys.size() != ref.size()) return std::fprintf(stderr, "walk size mismatch\n"), 1;
  size_t i = 0;
  for (const auto& it : ref)
    if (keys[i++] != it.first) return std::fprintf(stderr, "walk order mismatch\n"), 1;
  if (r.get("zzz_absent").first || r.get("").first || r.get("seq_").first)
    return std::fprintf(stderr, "absent key found\n"), 1;
  return 0;
}

static std::string slurp(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  std::string s;
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, n);
  std::fclose(f);
  return s;
}

static void spit(const std::string& path, const std::string& s) {
  FILE* f = std::fopen(path.c_str(), "wb");
  std::fwrite(s.data(), 1, s.size(), f);
  std::fclose(f);
}

int main(int argc, char** argv) {
  if (argc < 2) return std::fprintf(stderr, "usage: %s <scratch dir> [fuzz iterations]\n", argv[0]), 2;
  const std::string root = argv[1];
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  std::mt19937_64 rng(1234);
  int rc = 0;
  rc |= round_trip(root + "/small", rng, 300, 200, 4096);       // inline values, one leaf level
  rc |= round_trip(root + "/big", rng, 40, 30000, 4096);        // overflow pages
  rc |= round_trip(root + "/deep", rng, 20000, 64, 4096);       // multi-level branch tree
  rc |= round_trip(root + "/p8k", rng, 500, 9000, 8192);        // non-default page size
  if (rc) return rc;
  const std::string good = slurp(root + "/deep/data.mdb");
  const std::string good_big = slurp(root + "/big/data.mdb");
  ::mkdir((root + "/fuzz").c_str(), 0755);
  const std::string fz = root + "/fuzz/data.mdb";
  size_t opened = 0, thrown = 0;
  for (int it = 0; it < iters; ++it) {
    std::string s = (it & 1) ? good : good_big;
    const int mode = it % 3;
    if (mode == 0) {  // random byte flips
      const int n = 1 + static_cast<int>(rng() % 64);
      for (int k = 0; k < n; ++k) s[rng() % s.size()] ^= static_cast<char>(1 + rng() % 255);
    } else if (mode == 1) {  // truncation
      s.resize(rng() % s.size());
    } else {  // flips concentrated in the meta pages / first tree pages
      for (int k = 0; k < 8; ++k) s[rng() % std::min<size_t>(s.size(), 3 * 4096)] ^= (char)(rng() & 0xff);
    }
    spit(fz, s);
    try {
      Reader r(root + "/fuzz");
      ++opened;
      try {
        auto keys = r.keys();
        for (size_t k = 0; k < keys.size() && k < 64; ++k) {
          auto v = r.get(keys[k]);
          volatile char sink = 0;
          for (size_t b = 0; b < v.second; b += 97) sink ^= v.first[b];
          (void)sink;
        }
      } catch (const std::runtime_error&) {
        ++thrown;
      }
      r.get("seq_000010/frame_0001");
    } catch (const std::runtime_error&) {
      ++thrown;
    }
  }
  std::printf("lmdb sanitize: round trips ok; fuzz %d iterations, %zu opened, %zu rejected\n",
              iters, opened, thrown);
  return 0;
}
