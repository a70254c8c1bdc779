// TensorBoard event-file encoding (host runtime).
//
// The reference logs through SB3's TensorBoardOutputFormat (torch SummaryWriter), reached from
// imitation's HierarchicalLogger (src/imitation/util/logger.py:17-44); the CLI default formats
// are ["tensorboard", "stdout"] (src/imitation/scripts/ingredients/logging.py:35) and a GAIL round
// dumps 9 times (common.py:385, 461). Encoding those records in Python (protobuf varints +
// a CRC32C byte loop per record) cost more per round than the whole device GAIL round, so the
// records are built here: one call per dump encodes every scalar of the dump into framed
// TFRecords  [u64 length][u32 masked crc32c(length)][Event bytes][u32 masked crc32c(Event)].
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

namespace ia {
namespace {

struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    const uint32_t poly = 0x82F63B78u;  // Castagnoli, reflected
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ poly : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFFu];
  }
};

const Crc32cTables& tables() {
  static const Crc32cTables tb;
  return tb;
}

void put_varint(std::string& out, uint64_t v) {
  while (v >= 0x80) {
    out.push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  out.push_back((char)v);
}

void put_key(std::string& out, int field, int wire) { put_varint(out, ((uint64_t)field << 3) | (uint64_t)wire); }

template <typename T>
void put_le(std::string& out, T v) {
  char b[sizeof(T)];
  memcpy(b, &v, sizeof(T));  // little-endian host (x86-64 / gfx950 hosts)
  out.append(b, sizeof(T));
}

}  // namespace

// slicing-by-8 CRC32C (Castagnoli)
uint32_t crc32c(const uint8_t* p, size_t n) {
  const Crc32cTables& tb = tables();
  uint32_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = tb.t[7][lo & 0xFF] ^ tb.t[6][(lo >> 8) & 0xFF] ^ tb.t[5][(lo >> 16) & 0xFF] ^ tb.t[4][lo >> 24] ^
        tb.t[3][hi & 0xFF] ^ tb.t[2][(hi >> 8) & 0xFF] ^ tb.t[1][(hi >> 16) & 0xFF] ^ tb.t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = tb.t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

uint32_t masked_crc32c(const uint8_t* p, size_t n) {
  const uint32_t c = crc32c(p, n);
  return ((c >> 15) | (c << 17)) + 0xA282EAD8u;
}

// One framed TFRecord around `event`.
void tb_frame(std::string& out, const std::string& event) {
  std::string hdr;
  put_le<uint64_t>(hdr, (uint64_t)event.size());
  out += hdr;
  put_le<uint32_t>(out, masked_crc32c((const uint8_t*)hdr.data(), hdr.size()));
  out += event;
  put_le<uint32_t>(out, masked_crc32c((const uint8_t*)event.data(), event.size()));
}

// Event{wall_time, step, summary{value{tag, simple_value}}} per scalar, framed, concatenated.
std::string tb_scalar_records(double wall_time, int64_t step, const std::vector<std::string>& tags,
                              const std::vector<float>& values) {
  std::string out, ev, val, summ;
  out.reserve(tags.size() * 96);
  for (size_t i = 0; i < tags.size() && i < values.size(); ++i) {
    val.clear();
    put_key(val, 1, 2);
    put_varint(val, tags[i].size());
    val += tags[i];
    put_key(val, 2, 5);
    put_le<float>(val, values[i]);
    summ.clear();
    put_key(summ, 1, 2);
    put_varint(summ, val.size());
    summ += val;
    ev.clear();
    put_key(ev, 1, 1);
    put_le<double>(ev, wall_time);
    put_key(ev, 2, 0);
    put_varint(ev, (uint64_t)step);
    put_key(ev, 5, 2);
    put_varint(ev, summ.size());
    ev += summ;
    tb_frame(out, ev);
  }
  return out;
}

}  // namespace ia
