// TensorFlow tensor-bundle codec (see tf_bundle.h). Pure C++17, no TensorFlow / protobuf dependency.
#include "tf_bundle.h"

#include <algorithm>
#include <cstring>
#include <fstream>
#include <sstream>

namespace tfb {

// ------------------------------------------------------------------------------------------ CRC32C (Castagnoli)
static uint32_t g_table[8][256];
static bool g_init = false;

static void init_tables() {
  if (g_init) return;
  const uint32_t poly = 0x82F63B78u;  // reversed Castagnoli
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
    g_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) g_table[t][i] = (g_table[t - 1][i] >> 8) ^ g_table[0][g_table[t - 1][i] & 0xFF];
  g_init = true;
}

uint32_t crc32c(const uint8_t* p, size_t n, uint32_t init) {
  init_tables();
  uint32_t c = ~init;
  // slicing-by-8
  while (n >= 8) {
    uint32_t lo, hi;
    std::memcpy(&lo, p, 4);
    std::memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = g_table[7][lo & 0xFF] ^ g_table[6][(lo >> 8) & 0xFF] ^ g_table[5][(lo >> 16) & 0xFF] ^ g_table[4][lo >> 24] ^
        g_table[3][hi & 0xFF] ^ g_table[2][(hi >> 8) & 0xFF] ^ g_table[1][(hi >> 16) & 0xFF] ^ g_table[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ g_table[0][(c ^ *p++) & 0xFF];
  return ~c;
}

static const uint32_t kMaskDelta = 0xa282ead8u;
uint32_t mask_crc(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }
uint32_t unmask_crc(uint32_t m) {
  uint32_t rot = m - kMaskDelta;
  return (rot >> 17) | (rot << 15);
}

// ------------------------------------------------------------------------------------------ varints / fixed
static void put_varint(std::string* s, uint64_t v) {
  while (v >= 0x80) {
    s->push_back((char)((v & 0x7F) | 0x80));
    v >>= 7;
  }
  s->push_back((char)v);
}
static void put_fixed32(std::string* s, uint32_t v) {
  for (int i = 0; i < 4; ++i) s->push_back((char)((v >> (8 * i)) & 0xFF));
}
static void put_fixed64(std::string* s, uint64_t v) {
  for (int i = 0; i < 8; ++i) s->push_back((char)((v >> (8 * i)) & 0xFF));
}

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  Reader(const char* b, size_t n) : p((const uint8_t*)b), end((const uint8_t*)b + n) {}
  bool done() const { return p >= end; }
  uint64_t varint() {
    uint64_t r = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      if (p >= end) throw FormatError("truncated varint");
      const uint8_t b = *p++;
      r |= (uint64_t)(b & 0x7F) << shift;
      if (!(b & 0x80)) return r;
    }
    throw FormatError("varint too long");
  }
  uint32_t fixed32() {
    if (end - p < 4) throw FormatError("truncated fixed32");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) v |= (uint32_t)p[i] << (8 * i);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    uint64_t lo = fixed32();
    uint64_t hi = fixed32();
    return lo | (hi << 32);
  }
  std::string bytes(size_t n) {
    if ((size_t)(end - p) < n) throw FormatError("truncated bytes");
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
  void skip(int wire) {
    switch (wire) {
      case 0: varint(); break;
      case 1: bytes(8); break;
      case 2: bytes(varint()); break;
      case 5: bytes(4); break;
      default: throw FormatError("unsupported wire type");
    }
  }
};

// ------------------------------------------------------------------------------------------ protobuf messages
std::string encode_header(const Header& h) {
  std::string s;
  if (h.num_shards) { put_varint(&s, (1 << 3) | 0); put_varint(&s, (uint64_t)h.num_shards); }
  if (h.endianness) { put_varint(&s, (2 << 3) | 0); put_varint(&s, (uint64_t)h.endianness); }
  std::string ver;
  if (h.producer) { put_varint(&ver, (1 << 3) | 0); put_varint(&ver, (uint64_t)h.producer); }
  if (h.min_consumer) { put_varint(&ver, (2 << 3) | 0); put_varint(&ver, (uint64_t)h.min_consumer); }
  put_varint(&s, (3 << 3) | 2);
  put_varint(&s, ver.size());
  s += ver;
  return s;
}

Header decode_header(const std::string& v) {
  Header h;
  h.num_shards = 0;
  h.producer = 0;
  Reader r(v.data(), v.size());
  while (!r.done()) {
    const uint64_t tag = r.varint();
    const int field = (int)(tag >> 3), wire = (int)(tag & 7);
    if (field == 1 && wire == 0) h.num_shards = (int32_t)r.varint();
    else if (field == 2 && wire == 0) h.endianness = (int32_t)r.varint();
    else if (field == 3 && wire == 2) {
      std::string sub = r.bytes(r.varint());
      Reader q(sub.data(), sub.size());
      while (!q.done()) {
        const uint64_t t2 = q.varint();
        const int f2 = (int)(t2 >> 3), w2 = (int)(t2 & 7);
        if (f2 == 1 && w2 == 0) h.producer = (int32_t)q.varint();
        else if (f2 == 2 && w2 == 0) h.min_consumer = (int32_t)q.varint();
        else q.skip(w2);
      }
    } else r.skip(wire);
  }
  return h;
}

std::string encode_entry(const Entry& e) {
  std::string s;
  if (e.dtype) { put_varint(&s, (1 << 3) | 0); put_varint(&s, (uint64_t)e.dtype); }
  std::string shape;
  for (int64_t d : e.shape) {
    std::string dim;
    if (d) { put_varint(&dim, (1 << 3) | 0); put_varint(&dim, (uint64_t)d); }
    put_varint(&shape, (2 << 3) | 2);
    put_varint(&shape, dim.size());
    shape += dim;
  }
  put_varint(&s, (2 << 3) | 2);
  put_varint(&s, shape.size());
  s += shape;
  if (e.shard_id) { put_varint(&s, (3 << 3) | 0); put_varint(&s, (uint64_t)e.shard_id); }
  if (e.offset) { put_varint(&s, (4 << 3) | 0); put_varint(&s, (uint64_t)e.offset); }
  if (e.size) { put_varint(&s, (5 << 3) | 0); put_varint(&s, (uint64_t)e.size); }
  if (e.has_crc) { put_varint(&s, (6 << 3) | 5); put_fixed32(&s, e.crc32c); }
  return s;
}

Entry decode_entry(const std::string& key, const std::string& v) {
  Entry e;
  e.key = key;
  e.dtype = 0;
  e.has_crc = false;
  Reader r(v.data(), v.size());
  while (!r.done()) {
    const uint64_t tag = r.varint();
    const int field = (int)(tag >> 3), wire = (int)(tag & 7);
    if (field == 1 && wire == 0) e.dtype = (int)r.varint();
    else if (field == 2 && wire == 2) {
      std::string sub = r.bytes(r.varint());
      Reader q(sub.data(), sub.size());
      while (!q.done()) {
        const uint64_t t2 = q.varint();
        const int f2 = (int)(t2 >> 3), w2 = (int)(t2 & 7);
        if (f2 == 2 && w2 == 2) {
          std::string dim = q.bytes(q.varint());
          Reader dr(dim.data(), dim.size());
          int64_t size = 0;
          while (!dr.done()) {
            const uint64_t t3 = dr.varint();
            if ((t3 >> 3) == 1 && (t3 & 7) == 0) size = (int64_t)dr.varint();
            else dr.skip((int)(t3 & 7));
          }
          e.shape.push_back(size);
        } else q.skip(w2);
      }
    } else if (field == 3 && wire == 0) e.shard_id = (int32_t)r.varint();
    else if (field == 4 && wire == 0) e.offset = (int64_t)r.varint();
    else if (field == 5 && wire == 0) e.size = (int64_t)r.varint();
    else if (field == 6 && wire == 5) { e.crc32c = r.fixed32(); e.has_crc = true; }
    else r.skip(wire);
  }
  return e;
}

// ------------------------------------------------------------------------------------------ table blocks
namespace {

struct BlockBuilder {
  int restart_interval;
  std::string buf;
  std::vector<uint32_t> restarts{0};
  int counter = 0;
  std::string last_key;
  explicit BlockBuilder(int ri) : restart_interval(ri) {}
  bool empty() const { return buf.empty(); }
  size_t estimate() const { return buf.size() + restarts.size() * 4 + 4; }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter < restart_interval) {
      const size_t mn = std::min(last_key.size(), key.size());
      while (shared < mn && last_key[shared] == key[shared]) ++shared;
    } else {
      restarts.push_back((uint32_t)buf.size());
      counter = 0;
    }
    const size_t non_shared = key.size() - shared;
    put_varint(&buf, shared);
    put_varint(&buf, non_shared);
    put_varint(&buf, value.size());
    buf.append(key.data() + shared, non_shared);
    buf += value;
    last_key = key;
    ++counter;
  }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) put_fixed32(&out, r);
    put_fixed32(&out, (uint32_t)restarts.size());
    return out;
  }
};

// bytewise comparator helpers (leveldb/TF semantics)
void shortest_separator(std::string* start, const std::string& limit) {
  size_t mn = std::min(start->size(), limit.size());
  size_t diff = 0;
  while (diff < mn && (*start)[diff] == limit[diff]) ++diff;
  if (diff >= mn) return;  // one is a prefix of the other
  const uint8_t b = (uint8_t)(*start)[diff];
  if (b < 0xff && b + 1 < (uint8_t)limit[diff]) {
    (*start)[diff]++;
    start->resize(diff + 1);
  }
}

void short_successor(std::string* key) {
  for (size_t i = 0; i < key->size(); ++i) {
    const uint8_t b = (uint8_t)(*key)[i];
    if (b != 0xff) {
      (*key)[i] = (char)(b + 1);
      key->resize(i + 1);
      return;
    }
  }
}

void append_block(std::string* file, const std::string& block, uint64_t* off, uint64_t* size) {
  *off = file->size();
  *size = block.size();
  *file += block;
  std::string trailer;
  trailer.push_back('\0');  // kNoCompression
  uint32_t c = crc32c((const uint8_t*)block.data(), block.size());
  c = crc32c((const uint8_t*)trailer.data(), 1, c);
  put_fixed32(&trailer, mask_crc(c));
  *file += trailer;
}

std::string read_block(const std::string& file, uint64_t off, uint64_t size) {
  // (no off + size + 5 sum: handles come from the file and the sum can wrap around 64 bits -- found by the ASan
  // self-test, csrc/tfbundle/selftest.cpp)
  if (off > file.size() || size > file.size() - off || file.size() - off - size < 5)
    throw FormatError("block handle out of range");
  const std::string block = file.substr(off, size);
  const uint8_t type = (uint8_t)file[off + size];
  if (type != 0) throw FormatError("compressed blocks are not supported");
  Reader tr(file.data() + off + size + 1, 4);
  const uint32_t want = unmask_crc(tr.fixed32());
  uint32_t c = crc32c((const uint8_t*)block.data(), block.size());
  c = crc32c(&type, 1, c);
  if (c != want) throw FormatError("block checksum mismatch");
  return block;
}

void iterate_block(const std::string& block, std::vector<std::pair<std::string, std::string>>* out) {
  if (block.size() < 4) throw FormatError("block too small");
  Reader cnt(block.data() + block.size() - 4, 4);
  const uint32_t nrest = cnt.fixed32();
  if ((uint64_t)nrest * 4 + 4 > block.size()) throw FormatError("bad restart count");
  const size_t limit = block.size() - 4 - (size_t)nrest * 4;
  Reader r(block.data(), limit);
  std::string key;
  while (!r.done()) {
    const uint64_t shared = r.varint(), non_shared = r.varint(), vlen = r.varint();
    if (shared > key.size()) throw FormatError("bad key prefix");
    key.resize(shared);
    key += r.bytes(non_shared);
    out->emplace_back(key, r.bytes(vlen));
  }
}

const uint64_t kTableMagic = 0xdb4775248b80fb57ull;

}  // namespace

std::string build_index(const Header& header, const std::vector<Entry>& entries_in, int restart_interval,
                        size_t block_size) {
  std::vector<std::pair<std::string, std::string>> kv;
  kv.emplace_back("", encode_header(header));
  std::vector<Entry> entries = entries_in;
  std::sort(entries.begin(), entries.end(), [](const Entry& a, const Entry& b) { return a.key < b.key; });
  for (const Entry& e : entries) {
    if (e.key.empty()) throw FormatError("empty tensor name");
    kv.emplace_back(e.key, encode_entry(e));
  }
  std::string file;
  BlockBuilder data(restart_interval), index(1);
  std::string last_key;
  bool pending = false;
  uint64_t pend_off = 0, pend_size = 0;
  for (size_t i = 0; i < kv.size(); ++i) {
    const std::string& key = kv[i].first;
    if (pending) {
      std::string sep = last_key;
      shortest_separator(&sep, key);
      std::string h;
      put_varint(&h, pend_off);
      put_varint(&h, pend_size);
      index.add(sep, h);
      pending = false;
    }
    data.add(key, kv[i].second);
    last_key = key;
    if (data.estimate() >= block_size) {
      append_block(&file, data.finish(), &pend_off, &pend_size);
      data = BlockBuilder(restart_interval);
      pending = true;
    }
  }
  if (!data.empty()) {
    append_block(&file, data.finish(), &pend_off, &pend_size);
    pending = true;
  }
  if (pending) {
    std::string succ = last_key;
    short_successor(&succ);
    std::string h;
    put_varint(&h, pend_off);
    put_varint(&h, pend_size);
    index.add(succ, h);
  }
  uint64_t meta_off, meta_size, idx_off, idx_size;
  BlockBuilder meta(restart_interval);
  append_block(&file, meta.finish(), &meta_off, &meta_size);
  append_block(&file, index.finish(), &idx_off, &idx_size);
  std::string footer;
  put_varint(&footer, meta_off);
  put_varint(&footer, meta_size);
  put_varint(&footer, idx_off);
  put_varint(&footer, idx_size);
  footer.resize(40, '\0');
  put_fixed64(&footer, kTableMagic);
  file += footer;
  return file;
}

void parse_index(const std::string& file, Header* header, std::vector<Entry>* entries) {
  if (file.size() < 48) throw FormatError("index file too small");
  Reader fr(file.data() + file.size() - 48, 48);
  const uint64_t meta_off = fr.varint(), meta_size = fr.varint();
  const uint64_t idx_off = fr.varint(), idx_size = fr.varint();
  (void)meta_off;
  (void)meta_size;
  Reader mr(file.data() + file.size() - 8, 8);
  if (mr.fixed64() != kTableMagic) throw FormatError("bad table magic");
  const std::string idx = read_block(file, idx_off, idx_size);
  std::vector<std::pair<std::string, std::string>> handles;
  iterate_block(idx, &handles);
  bool have_header = false;
  for (auto& kvh : handles) {
    Reader hr(kvh.second.data(), kvh.second.size());
    const uint64_t off = hr.varint(), size = hr.varint();
    std::vector<std::pair<std::string, std::string>> kv;
    iterate_block(read_block(file, off, size), &kv);
    for (auto& e : kv) {
      if (e.first.empty()) {
        *header = decode_header(e.second);
        have_header = true;
      } else {
        entries->push_back(decode_entry(e.first, e.second));
      }
    }
  }
  if (!have_header) throw FormatError("missing bundle header");
}

size_t dtype_size(int dtype) {
  switch (dtype) {
    case 1: return 4;    // float
    case 2: return 8;    // double
    case 3: return 4;    // int32
    case 4: return 1;    // uint8
    case 5: return 2;    // int16
    case 6: return 1;    // int8
    case 9: return 8;    // int64
    case 10: return 1;   // bool
    case 14: return 2;   // bfloat16
    case 17: return 2;   // uint16
    case 19: return 2;   // half
    case 22: return 4;   // uint32
    case 23: return 8;   // uint64
    default: throw FormatError("unsupported dtype " + std::to_string(dtype));
  }
}

static std::string data_path(const std::string& prefix, int shard = 0, int nshards = 1) {
  char buf[64];
  std::snprintf(buf, sizeof(buf), ".data-%05d-of-%05d", shard, nshards);
  return prefix + buf;
}

static std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

void write_bundle(const std::string& prefix, std::vector<Tensor> tensors) {
  std::sort(tensors.begin(), tensors.end(), [](const Tensor& a, const Tensor& b) { return a.key < b.key; });
  std::vector<Entry> entries;
  std::string data;
  for (size_t i = 0; i < tensors.size(); ++i) {
    const Tensor& t = tensors[i];
    if (i && tensors[i - 1].key == t.key) throw FormatError("duplicate tensor name " + t.key);
    int64_t n = 1;
    for (int64_t d : t.shape) n *= d;
    if ((int64_t)t.data.size() != n * (int64_t)dtype_size(t.dtype))
      throw FormatError("tensor " + t.key + ": byte size does not match shape");
    Entry e;
    e.key = t.key;
    e.dtype = t.dtype;
    e.shape = t.shape;
    e.offset = (int64_t)data.size();
    e.size = (int64_t)t.data.size();
    e.crc32c = mask_crc(crc32c((const uint8_t*)t.data.data(), t.data.size()));
    entries.push_back(e);
    data += t.data;
  }
  Header h;
  const std::string index = build_index(h, entries);
  {
    std::ofstream f(data_path(prefix), std::ios::binary | std::ios::trunc);
    if (!f) throw std::runtime_error("cannot write " + data_path(prefix));
    f.write(data.data(), data.size());
  }
  {
    std::ofstream f(prefix + ".index", std::ios::binary | std::ios::trunc);
    if (!f) throw std::runtime_error("cannot write " + prefix + ".index");
    f.write(index.data(), index.size());
  }
}

std::vector<Tensor> read_bundle(const std::string& prefix, bool verify_crc) {
  Header h;
  std::vector<Entry> entries;
  parse_index(slurp(prefix + ".index"), &h, &entries);
  if (h.endianness != 0) throw FormatError("big-endian bundles are not supported");
  if (h.num_shards < 0 || h.num_shards > 65536) throw FormatError("bad shard count");
  std::vector<std::string> shards;
  for (int s = 0; s < std::max(1, h.num_shards); ++s) shards.push_back(slurp(data_path(prefix, s, h.num_shards)));
  std::vector<Tensor> out;
  for (const Entry& e : entries) {
    if (e.shard_id < 0 || e.shard_id >= (int)shards.size()) throw FormatError("bad shard id for " + e.key);
    const std::string& d = shards[e.shard_id];
    if (e.offset < 0 || e.size < 0 || (uint64_t)e.offset > d.size() || (uint64_t)e.size > d.size() - (uint64_t)e.offset)
      throw FormatError("tensor " + e.key + " out of range of the data file");
    Tensor t;
    t.key = e.key;
    t.dtype = e.dtype;
    t.shape = e.shape;
    t.data = d.substr(e.offset, e.size);
    if (verify_crc && e.has_crc) {
      const uint32_t c = mask_crc(crc32c((const uint8_t*)t.data.data(), t.data.size()));
      if (c != e.crc32c) throw FormatError("checksum mismatch for tensor " + e.key);
    }
    out.push_back(std::move(t));
  }
  return out;
}

}  // namespace tfb
