// TensorFlow "V2" checkpoint (tensor bundle) writer and reader.
//
// What the reference's FastSaver (utils.py:28-32, a tf.train.Saver with
// write_meta_graph=False) produces through TF's C++ SaveV2 op, and what the
// Supervisor restores on chief start (worker.py:107-118):
//
//   <prefix>.data-00000-of-00001   raw little-endian tensor bytes, back to back
//   <prefix>.index                 an SSTable (LevelDB table format):
//       key ""          -> BundleHeaderProto{num_shards=1, endianness=LITTLE,
//                                            version{producer=1}}
//       key <var name>  -> BundleEntryProto{dtype, shape, shard_id, offset,
//                                           size, crc32c = masked CRC32C}
//       data blocks (prefix-compressed entries, restart points every 16)
//       + empty metaindex block + index block + 48-byte footer
//         (two varint BlockHandles padded to 40 bytes, magic 0xdb4775248b80fb57)
//       every block followed by [type byte 0 = no compression][masked crc32c]
//
// Keys are written in bytewise order (the table is sorted); tensor data in
// the same order, no alignment padding (BundleWriter's default).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "crc32c.h"
#include "proto.h"

namespace py = pybind11;
using namespace dtfx_host;

namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;
constexpr size_t kBlockSize = 262144;  // table::Options default block_size
constexpr int kRestartInterval = 16;   // table::Options default block_restart_interval
constexpr size_t kFooterLen = 48;

// TF DataType enum values
enum DType : int { DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_UINT8 = 4, DT_INT16 = 5,
                   DT_INT8 = 6, DT_INT64 = 9, DT_BOOL = 10, DT_BFLOAT16 = 14, DT_HALF = 19 };

size_t dtype_size(int dt) {
  switch (dt) {
    case DT_FLOAT: case DT_INT32: return 4;
    case DT_DOUBLE: case DT_INT64: return 8;
    case DT_UINT8: case DT_INT8: case DT_BOOL: return 1;
    case DT_INT16: case DT_BFLOAT16: case DT_HALF: return 2;
    default: throw std::runtime_error("tensor_bundle: unsupported dtype " + std::to_string(dt));
  }
}

struct BlockBuilder {
  std::string buf;
  std::vector<uint32_t> restarts{0};
  int counter = 0;
  std::string last_key;
  bool empty() const { return buf.empty(); }
  size_t estimate() const { return buf.size() + restarts.size() * 4 + 4; }
  void add(const std::string& key, const std::string& value) {
    size_t shared = 0;
    if (counter < kRestartInterval) {
      const size_t mn = std::min(last_key.size(), key.size());
      while (shared < mn && last_key[shared] == key[shared]) ++shared;
    } else {
      restarts.push_back(static_cast<uint32_t>(buf.size()));
      counter = 0;
    }
    pb::put_varint(buf, shared);
    pb::put_varint(buf, key.size() - shared);
    pb::put_varint(buf, value.size());
    buf.append(key, shared, std::string::npos);
    buf.append(value);
    last_key = key;
    ++counter;
  }
  std::string finish() {
    std::string out = buf;
    for (uint32_t r : restarts) pb::put_fixed32(out, r);
    pb::put_fixed32(out, static_cast<uint32_t>(restarts.size()));
    return out;
  }
  void reset() {
    buf.clear();
    restarts.assign(1, 0);
    counter = 0;
    last_key.clear();
  }
};

// LevelDB BytewiseComparator::FindShortestSeparator / FindShortSuccessor
void shortest_separator(std::string* start, const std::string& limit) {
  const size_t mn = std::min(start->size(), limit.size());
  size_t d = 0;
  while (d < mn && (*start)[d] == limit[d]) ++d;
  if (d >= mn) return;
  const uint8_t b = static_cast<uint8_t>((*start)[d]);
  if (b < 0xff && b + 1 < static_cast<uint8_t>(limit[d])) {
    (*start)[d] = static_cast<char>(b + 1);
    start->resize(d + 1);
  }
}
void short_successor(std::string* key) {
  for (size_t i = 0; i < key->size(); ++i) {
    const uint8_t b = static_cast<uint8_t>((*key)[i]);
    if (b != 0xff) {
      (*key)[i] = static_cast<char>(b + 1);
      key->resize(i + 1);
      return;
    }
  }
}

struct TableWriter {
  std::string file;  // whole table in memory (index files are tiny)
  BlockBuilder data, index;
  std::string last_key;
  bool pending_index = false;
  uint64_t pend_off = 0, pend_size = 0;

  static std::string handle(uint64_t off, uint64_t size) {
    std::string h;
    pb::put_varint(h, off);
    pb::put_varint(h, size);
    return h;
  }
  void write_block(const std::string& contents, uint64_t* off, uint64_t* size) {
    *off = file.size();
    *size = contents.size();
    file.append(contents);
    const char type = 0;  // kNoCompression
    uint32_t crc = crc32c(contents.data(), contents.size());
    crc = crc32c_extend(crc, &type, 1);
    file.push_back(type);
    pb::put_fixed32(file, crc32c_mask(crc));
  }
  void flush_data() {
    if (data.empty()) return;
    write_block(data.finish(), &pend_off, &pend_size);
    data.reset();
    pending_index = true;
  }
  void add(const std::string& key, const std::string& value) {
    if (!last_key.empty() || !file.empty() || !data.empty())
      if (key < last_key) throw std::runtime_error("tensor_bundle: keys must be added in order");
    if (pending_index) {
      std::string sep = last_key;
      shortest_separator(&sep, key);
      index.add(sep, handle(pend_off, pend_size));
      pending_index = false;
    }
    data.add(key, value);
    last_key = key;
    if (data.estimate() >= kBlockSize) flush_data();
  }
  std::string finish() {
    flush_data();
    uint64_t meta_off, meta_size;
    BlockBuilder meta;
    write_block(meta.finish(), &meta_off, &meta_size);
    if (pending_index) {
      std::string succ = last_key;
      short_successor(&succ);
      index.add(succ, handle(pend_off, pend_size));
      pending_index = false;
    }
    uint64_t idx_off, idx_size;
    write_block(index.finish(), &idx_off, &idx_size);
    std::string footer = handle(meta_off, meta_size) + handle(idx_off, idx_size);
    footer.resize(40, '\0');
    pb::put_fixed64(footer, kTableMagic);
    file.append(footer);
    return file;
  }
};

// --------------------------------------------------------------------------
// table reading
// --------------------------------------------------------------------------
std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

std::string block_at(const std::string& file, uint64_t off, uint64_t size, bool verify) {
  if (off + size + 5 > file.size()) throw std::runtime_error("sstable: block out of range");
  std::string contents = file.substr(off, size);
  if (verify) {
    const char type = file[off + size];
    if (type != 0) throw std::runtime_error("sstable: compressed blocks are not supported");
    uint32_t crc = crc32c(contents.data(), contents.size());
    crc = crc32c_extend(crc, &type, 1);
    uint32_t stored;
    std::memcpy(&stored, file.data() + off + size + 1, 4);
    if (crc32c_unmask(stored) != crc) throw std::runtime_error("sstable: block checksum mismatch");
  }
  return contents;
}

std::vector<std::pair<std::string, std::string>> block_entries(const std::string& blk) {
  if (blk.size() < 4) throw std::runtime_error("sstable: short block");
  uint32_t nrest;
  std::memcpy(&nrest, blk.data() + blk.size() - 4, 4);
  const size_t limit = blk.size() - 4 - 4ull * nrest;
  if (limit > blk.size()) throw std::runtime_error("sstable: bad restart array");
  std::vector<std::pair<std::string, std::string>> out;
  pb::Reader r(blk.data(), limit);
  std::string key;
  while (!r.done()) {
    const uint64_t shared = r.varint(), nonshared = r.varint(), vlen = r.varint();
    if (shared > key.size() || static_cast<uint64_t>(r.end - r.p) < nonshared + vlen)
      throw std::runtime_error("sstable: corrupt entry");
    key.resize(shared);
    key.append(reinterpret_cast<const char*>(r.p), nonshared);
    r.p += nonshared;
    std::string value(reinterpret_cast<const char*>(r.p), vlen);
    r.p += vlen;
    out.emplace_back(key, value);
  }
  return out;
}

std::vector<std::pair<std::string, std::string>> read_table(const std::string& file, bool verify) {
  if (file.size() < kFooterLen) throw std::runtime_error("sstable: file too short");
  const std::string footer = file.substr(file.size() - kFooterLen);
  uint64_t magic;
  std::memcpy(&magic, footer.data() + 40, 8);
  if (magic != kTableMagic) throw std::runtime_error("sstable: bad magic (not a TF table)");
  pb::Reader fr(footer.data(), 40);
  fr.varint();
  fr.varint();  // metaindex handle (unused)
  const uint64_t ioff = fr.varint(), isize = fr.varint();
  std::vector<std::pair<std::string, std::string>> out;
  for (auto& ie : block_entries(block_at(file, ioff, isize, verify))) {
    pb::Reader hr(ie.second);
    const uint64_t off = hr.varint(), size = hr.varint();
    for (auto& kv : block_entries(block_at(file, off, size, verify))) out.push_back(kv);
  }
  return out;
}

// --------------------------------------------------------------------------
// protos
// --------------------------------------------------------------------------
std::string header_proto(int num_shards) {
  std::string h;
  pb::put_varint_field(h, 1, num_shards);  // num_shards
  // endianness LITTLE = 0: proto3 default, omitted
  std::string ver;
  pb::put_varint_field(ver, 1, 1);  // producer = kTensorBundleVersion (1)
  pb::put_bytes_field(h, 3, ver);
  return h;
}

std::string entry_proto(int dtype, const std::vector<int64_t>& shape, int shard, uint64_t offset,
                        uint64_t size, uint32_t masked_crc) {
  std::string e;
  pb::put_varint_field(e, 1, dtype);
  std::string sh;
  for (int64_t d : shape) {
    std::string dim;
    if (d != 0) pb::put_varint_field(dim, 1, static_cast<uint64_t>(d));
    pb::put_bytes_field(sh, 2, dim);
  }
  pb::put_bytes_field(e, 2, sh);
  if (shard) pb::put_varint_field(e, 3, shard);
  if (offset) pb::put_varint_field(e, 4, offset);
  if (size) pb::put_varint_field(e, 5, size);
  pb::put_fixed32_field(e, 6, masked_crc);
  return e;
}

struct Entry {
  int dtype = 0;
  std::vector<int64_t> shape;
  int shard = 0;
  uint64_t offset = 0, size = 0;
  uint32_t crc = 0;
};

Entry parse_entry(const std::string& v) {
  Entry e;
  pb::Reader r(v);
  while (!r.done()) {
    const uint64_t tag = r.varint();
    const uint32_t f = tag >> 3, w = tag & 7;
    if (f == 1 && w == 0) e.dtype = static_cast<int>(r.varint());
    else if (f == 2 && w == 2) {
      const std::string sbuf = r.bytes();
      pb::Reader sr(sbuf);
      while (!sr.done()) {
        const uint64_t st = sr.varint();
        if ((st >> 3) == 2 && (st & 7) == 2) {
          const std::string dbuf = sr.bytes();
          pb::Reader dr(dbuf);
          int64_t size = 0;
          while (!dr.done()) {
            const uint64_t dt = dr.varint();
            if ((dt >> 3) == 1 && (dt & 7) == 0) size = static_cast<int64_t>(dr.varint());
            else dr.skip(dt & 7);
          }
          e.shape.push_back(size);
        } else sr.skip(st & 7);
      }
    } else if (f == 3 && w == 0) e.shard = static_cast<int>(r.varint());
    else if (f == 4 && w == 0) e.offset = r.varint();
    else if (f == 5 && w == 0) e.size = r.varint();
    else if (f == 6 && w == 5) e.crc = r.fixed32();
    else if (f == 7) throw std::runtime_error("tensor_bundle: sliced tensors are not supported");
    else r.skip(w);
  }
  return e;
}

// --------------------------------------------------------------------------
// python API
// --------------------------------------------------------------------------
// write_bundle(prefix, [(name, dtype, shape, bytes)], ) -> None
void write_bundle(const std::string& prefix, py::list tensors) {
  struct T { std::string name; int dtype; std::vector<int64_t> shape; std::string data; };
  std::vector<T> ts;
  for (auto item : tensors) {
    auto tup = item.cast<py::tuple>();
    T t{tup[0].cast<std::string>(), tup[1].cast<int>(), tup[2].cast<std::vector<int64_t>>(),
        tup[3].cast<std::string>()};
    size_t n = 1;
    for (int64_t d : t.shape) n *= static_cast<size_t>(d);
    if (n * dtype_size(t.dtype) != t.data.size())
      throw std::runtime_error("tensor_bundle: byte size mismatch for " + t.name);
    ts.push_back(std::move(t));
  }
  std::sort(ts.begin(), ts.end(), [](const T& a, const T& b) { return a.name < b.name; });
  for (size_t i = 1; i < ts.size(); ++i)
    if (ts[i].name == ts[i - 1].name) throw std::runtime_error("duplicate tensor " + ts[i].name);
  const std::string data_path = prefix + ".data-00000-of-00001";
  const std::string tmp_data = data_path + ".tempstate", tmp_index = prefix + ".index.tempstate";
  TableWriter tw;
  tw.add("", header_proto(1));
  {
    std::ofstream df(tmp_data, std::ios::binary | std::ios::trunc);
    if (!df) throw std::runtime_error("cannot write " + tmp_data);
    uint64_t off = 0;
    for (auto& t : ts) {
      df.write(t.data.data(), static_cast<std::streamsize>(t.data.size()));
      const uint32_t crc = crc32c(t.data.data(), t.data.size());
      tw.add(t.name, entry_proto(t.dtype, t.shape, 0, off, t.data.size(), crc32c_mask(crc)));
      off += t.data.size();
    }
    if (!df) throw std::runtime_error("write failed: " + tmp_data);
  }
  {
    const std::string idx = tw.finish();
    std::ofstream f(tmp_index, std::ios::binary | std::ios::trunc);
    f.write(idx.data(), static_cast<std::streamsize>(idx.size()));
    if (!f) throw std::runtime_error("write failed: " + tmp_index);
  }
  // atomic publish, data first (TF renames the same way)
  if (std::rename(tmp_data.c_str(), data_path.c_str()) != 0 ||
      std::rename(tmp_index.c_str(), (prefix + ".index").c_str()) != 0)
    throw std::runtime_error("rename failed for checkpoint " + prefix);
}

// read_bundle(prefix) -> {name: (dtype, shape, bytes)}
py::dict read_bundle(const std::string& prefix, bool verify) {
  const std::string idx = read_file(prefix + ".index");
  auto entries = read_table(idx, verify);
  if (entries.empty() || !entries[0].first.empty())
    throw std::runtime_error("tensor_bundle: missing header entry");
  int num_shards = 1;
  {
    pb::Reader r(entries[0].second);
    while (!r.done()) {
      const uint64_t tag = r.varint();
      if ((tag >> 3) == 1 && (tag & 7) == 0) num_shards = static_cast<int>(r.varint());
      else if ((tag >> 3) == 2 && (tag & 7) == 0) {
        if (r.varint() != 0) throw std::runtime_error("tensor_bundle: big-endian bundles unsupported");
      } else r.skip(tag & 7);
    }
  }
  std::vector<std::string> shards(num_shards);
  py::dict out;
  for (size_t i = 1; i < entries.size(); ++i) {
    Entry e = parse_entry(entries[i].second);
    if (e.shard < 0 || e.shard >= num_shards) throw std::runtime_error("bad shard id");
    if (shards[e.shard].empty()) {
      char name[64];
      std::snprintf(name, sizeof(name), ".data-%05d-of-%05d", e.shard, num_shards);
      shards[e.shard] = read_file(prefix + name);
    }
    const std::string& d = shards[e.shard];
    if (e.offset + e.size > d.size()) throw std::runtime_error("tensor_bundle: data out of range");
    std::string bytes = d.substr(e.offset, e.size);
    if (verify && crc32c_unmask(e.crc) != crc32c(bytes.data(), bytes.size()))
      throw std::runtime_error("tensor_bundle: data checksum mismatch for " + entries[i].first);
    out[py::str(entries[i].first)] = py::make_tuple(e.dtype, e.shape, py::bytes(bytes));
  }
  return out;
}

}  // namespace

void register_bundle(py::module_& m) {
  m.def("write_bundle", &write_bundle, py::arg("prefix"), py::arg("tensors"),
        "Write a TF V2 checkpoint: list of (name, tf_dtype, shape, raw_bytes).");
  m.def("read_bundle", &read_bundle, py::arg("prefix"), py::arg("verify") = true,
        "Read a TF V2 checkpoint -> {name: (tf_dtype, shape, raw_bytes)}.");
  m.def("read_table", [](py::bytes b, bool verify) {
    std::string s = b;
    py::list out;
    for (auto& kv : read_table(s, verify)) out.append(py::make_tuple(py::bytes(kv.first), py::bytes(kv.second)));
    return out;
  }, py::arg("data"), py::arg("verify") = true, "Decode an SSTable (LevelDB format) -> [(key, value)].");
  m.def("build_table", [](py::list kvs) {
    TableWriter tw;
    for (auto item : kvs) {
      auto t = item.cast<py::tuple>();
      tw.add(t[0].cast<std::string>(), t[1].cast<std::string>());
    }
    return py::bytes(tw.finish());
  }, "Encode sorted (key, value) pairs as an SSTable.");
}
