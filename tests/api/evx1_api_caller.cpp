// tests/api/evx1_api_caller.cpp -- a C++ caller of the drop-in encoder,
// built against include/evx1.h exactly as a user of the reference would be
// (reference evx1.h:66-94, evx1.cpp:8-63, bitstream.h:43-92): it creates the
// encoder through evx::create_encoder, calls set_quality / encode through the
// evx1_encoder vtable, and reads the stream through bit_stream.
//
//   evx1_api_caller W H RING QUALITY FRAMES [--intra-every K] [--records FILE]
//
// Frames are band4 content, generated on the host before
// each call.  Prints one JSON line: per-call encode() wall time (ms), the bits
// of every frame record, and the FNV-1a-64 of the masked records (header byte
// 7 and the tail bits of each record's last byte zeroed: SURVEY.md
// Appendix A) -- the same canonical hash as tests/golden/oracle_streams.json.
// --records writes the raw records (u32 nbits + bytes per frame) for tests.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cairo_amd.h"
#include "../../include/evx1.h"

static uint64_t fnv1a64(uint64_t h, const uint8_t* d, size_t n) {
  for (size_t i = 0; i < n; i++) {
    h ^= d[i];
    h *= 0x100000001B3ull;
  }
  return h;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s W H RING QUALITY FRAMES [--intra-every K] [--records FILE]\n", argv[0]);
    return 2;
  }
  const uint32_t w = (uint32_t)atoi(argv[1]), h = (uint32_t)atoi(argv[2]);
  const uint32_t ring = (uint32_t)atoi(argv[3]);
  const int quality = atoi(argv[4]), frames = atoi(argv[5]);
  int intra_every = 0;
  const char* records = nullptr;
  for (int i = 6; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--intra-every")) intra_every = atoi(argv[i + 1]);
    if (!strcmp(argv[i], "--records")) records = argv[i + 1];
  }
  evx::evx1_encoder* enc = nullptr;
  if (evx::create_encoder(&enc) != EVX_SUCCESS) return 3;
  // R is compile-time in the reference (config.h:39); this library's C
  // extension sets it before the first frame
  if (ring != 4 && evx_encoder_set_ring(enc, ring) != 0) return 3;
  enc->set_quality((evx::uint8)quality);
  evx::bit_stream bs(w * h * 64 + 65536);
  std::vector<uint8_t> rgb((size_t)w * h * 3);
  std::vector<double> ms;
  std::vector<uint32_t> bits;
  uint64_t hash = 0xCBF29CE484222325ull;
  FILE* rec = records ? fopen(records, "wb") : nullptr;
  for (int t = 0; t < frames; t++) {
    cairo_make_band4(rgb.data(), w, h, (uint32_t)t, 1234);
    if (intra_every && t % intra_every == 0) enc->insert_intra();
    bs.empty();
    const auto t0 = std::chrono::steady_clock::now();
    const evx::evx_status st = enc->encode(rgb.data(), w, h, &bs);
    const auto t1 = std::chrono::steady_clock::now();
    if (st != EVX_SUCCESS) {
      fprintf(stderr, "encode failed on frame %d: status %d\n", t, (int)st);
      return 4;
    }
    ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
    const uint32_t n = bs.query_occupancy();
    bits.push_back(n);
    std::vector<uint8_t> b(bs.query_data(), bs.query_data() + (n + 7) / 8);
    if (rec) {
      fwrite(&n, 4, 1, rec);
      fwrite(b.data(), 1, b.size(), rec);
    }
    if (n % 8) b.back() &= (uint8_t)((1u << (n % 8)) - 1);
    if (t == 0 && b.size() > 7) b[7] = 0;
    hash = fnv1a64(hash, b.data(), b.size());
  }
  if (rec) fclose(rec);
  evx::destroy_encoder(enc);
  std::string out = "{\"encode_ms\": [";
  for (size_t i = 0; i < ms.size(); i++) out += (i ? ", " : "") + std::to_string(ms[i]);
  out += "], \"frame_bits\": [";
  for (size_t i = 0; i < bits.size(); i++) out += (i ? ", " : "") + std::to_string(bits[i]);
  char hx[32];
  snprintf(hx, sizeof(hx), "%016llx", (unsigned long long)hash);
  out += "], \"fnv1a64\": \"" + std::string(hx) + "\"}";
  printf("%s\n", out.c_str());
  return 0;
}
