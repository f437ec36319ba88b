// harp_amd/nc4read.hpp -- header-only reader of netCDF-4 files (HDF5 containers)
// for the RFM opacity tables and ck weights harp opens with
// nc_open(path, NC_NETCDF4, ...) and reads with nc_inq_dimid / nc_inq_dimlen /
// nc_inq_varid / nc_get_var_double (src/opacity/rfm.cpp:34-120,
// src/utils/read_weights.cpp:18-46).  Neither the netCDF nor the HDF5 library is
// a dependency: this walks the HDF5 file format (specification version 3) for
// what netCDF-4 writes into a flat root group --
//   superblock versions 0-3 (userblocks skipped),
//   object headers v1 and v2 with continuation blocks,
//   groups as symbol tables (v1 B-tree + local heap), compact link messages, or
//   dense links (fractal heap with direct/indirect blocks, v2 B-tree name index),
//   datasets: dataspace, fixed-point / IEEE float datatypes of either byte order,
//   compact / contiguous / chunked layouts (layout v3: v1 B-tree chunk index;
//   layout v4: single-chunk, implicit and fixed-array indexes),
//   filters: deflate (zlib), shuffle, fletcher32; fill value for unallocated chunks.
// A netCDF-4 dimension is a dataset of the same name (the coordinate variable,
// or netCDF's dimension-only scale), so dim_len(name) = that dataset's first
// extent.  Link with -lz.  Mirrored for Python by pyharp_amd/ncread.py through
// include/hdnc.h.
#pragma once

#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>
#include <iterator>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace harp_amd {

class NetCDF4 {
 public:
  // structural bounds of a file this reader trusts (user-supplied files: a cycle
  // of continuation blocks or B-tree children must end in an error, not a hang)
  static constexpr size_t kMaxBlocks = 4096;  // object-header continuation blocks
  static constexpr int kMaxDepth = 64;       // B-tree levels
  struct Dataset {
    std::vector<uint64_t> dims;
    int tclass = -1;  // 0 fixed point, 1 float
    int tsize = 0;
    bool big = false, sign = true;
    int layout = -1;  // 0 compact, 1 contiguous, 2 chunked
    int layout_version = 0;
    uint64_t addr = ~0ull, size = 0;  // contiguous / compact data / chunk-index address
    size_t compact_at = 0;
    std::vector<uint64_t> chunk;  // chunk dims (rank) ; element size dropped
    int index_type = 0;           // layout v4 chunk index (1 single, 2 implicit, 3 fixed array)
    uint64_t single_size = 0;
    uint32_t single_mask = 0;
    bool single_filtered = false;
    std::vector<std::pair<int, std::vector<uint32_t>>> filters;  // (id, client data)
    std::vector<uint8_t> fill;
  };

  explicit NetCDF4(std::string const& path) : path_(path) {
    std::ifstream f(path, std::ios::binary);
    if (!f.good()) throw std::runtime_error("nc4read: cannot open " + path);
    buf_.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    superblock();
    read_group(root_);
  }

  static bool is_hdf5(std::string const& path) {
    std::ifstream f(path, std::ios::binary);
    char s[8] = {0};
    f.read(s, 8);
    return f.gcount() == 8 && std::memcmp(s, kSig, 8) == 0;
  }

  //! nc_inq_dimid + nc_inq_dimlen: the first extent of the dataset named `name`
  size_t dim_len(std::string const& name) const {
    auto it = links_.find(name);
    if (it == links_.end())
      throw std::runtime_error(path_ + ": NetCDF: Invalid dimension ID or name (" + name + ")");
    Dataset d = dataset(it->second);
    return d.dims.empty() ? 1 : (size_t)d.dims[0];
  }

  std::vector<size_t> shape(std::string const& name) const {
    Dataset d = dataset(lookup(name));
    return std::vector<size_t>(d.dims.begin(), d.dims.end());
  }

  //! nc_inq_varid + nc_get_var_double: the whole variable, C order, as double
  std::vector<double> var(std::string const& name) const {
    Dataset d = dataset(lookup(name));
    std::vector<uint8_t> raw = read_raw(d);
    const size_t n = raw.size() / d.tsize;
    std::vector<double> out(n);
    for (size_t i = 0; i < n; ++i) out[i] = convert(d, raw.data() + i * d.tsize);
    return out;
  }

  std::vector<std::string> names() const {
    std::vector<std::string> v;
    for (auto const& kv : links_) v.push_back(kv.first);
    return v;
  }

 private:
  static constexpr char kSig[9] = "\x89HDF\r\n\x1a\n";
  std::string path_;
  std::vector<uint8_t> buf_;
  int so_ = 8, sl_ = 8;  // sizes of offsets and lengths
  uint64_t base_ = 0, root_ = 0;
  std::map<std::string, uint64_t> links_;  // root-group link -> object header address

  [[noreturn]] void bad(std::string const& what) const {
    throw std::runtime_error(path_ + ": netCDF-4/HDF5: " + what);
  }
  void need(uint64_t at, uint64_t n) const {
    if (at > buf_.size() || n > buf_.size() - at) bad("truncated file or bad address");
  }
  uint64_t le(uint64_t at, int n) const {
    need(at, n);
    uint64_t x = 0;
    for (int i = n - 1; i >= 0; --i) x = (x << 8) | buf_[at + i];
    return x;
  }
  bool undef(uint64_t a) const { return so_ == 8 ? a == ~0ull : a == ((1ull << (8 * so_)) - 1); }
  uint64_t abs_(uint64_t a) const { return base_ + a; }
  bool sig(uint64_t at, const char* s) const {
    need(at, 4);
    return std::memcmp(&buf_[at], s, 4) == 0;
  }

  // ---- superblock -----------------------------------------------------------
  void superblock() {
    uint64_t at = 0;
    for (;; at = at ? 2 * at : 512) {
      if (at + 8 > buf_.size()) bad("no HDF5 signature");
      if (std::memcmp(&buf_[at], kSig, 8) == 0) break;
    }
    const int v = buf_.at(at + 8);
    if (v == 0 || v == 1) {
      so_ = buf_.at(at + 13);
      sl_ = buf_.at(at + 14);
      uint64_t p = at + 24 + (v == 1 ? 4 : 0);
      base_ = le(p, so_);
      p += 4 * so_;            // base, free-space, end-of-file, driver info
      root_ = le(p + so_, so_);  // root symbol-table entry: name offset, header address
    } else if (v == 2 || v == 3) {
      so_ = buf_.at(at + 9);
      sl_ = buf_.at(at + 10);
      uint64_t p = at + 12;
      base_ = le(p, so_);
      root_ = le(p + 3 * so_, so_);  // base, extension, end-of-file, root header
    } else {
      bad("superblock version " + std::to_string(v));
    }
    if (so_ != 2 && so_ != 4 && so_ != 8) bad("size of offsets");
  }

  // ---- object headers -------------------------------------------------------
  struct Msg {
    int type;
    uint64_t at;  // absolute offset of the message data
    uint64_t size;
  };

  std::vector<Msg> messages(uint64_t addr) const {
    std::vector<Msg> out;
    const uint64_t a = abs_(addr);
    need(a, 16);
    if (sig(a, "OHDR")) {
      const int flags = buf_[a + 5];
      uint64_t p = a + 6;
      if (flags & 0x20) p += 16;
      if (flags & 0x10) p += 4;
      const int w = 1 << (flags & 3);
      const uint64_t sz = le(p, w);
      p += w;
      std::vector<std::pair<uint64_t, uint64_t>> blocks{{p, p + sz}};
      for (size_t b = 0; b < blocks.size(); ++b) {
        if (b >= kMaxBlocks) bad("object header: too many continuation blocks (cycle?)");
        uint64_t q = blocks[b].first;
        const uint64_t end = blocks[b].second;
        const int hdr = (flags & 0x04) ? 6 : 4;
        while (q + hdr <= end) {
          const int type = buf_[q];
          const uint64_t size = le(q + 1, 2);
          const uint64_t d = q + hdr;
          need(d, size);
          if (type == 0x10) {
            const uint64_t off = abs_(le(d, so_)), len = le(d + so_, sl_);
            if (!sig(off, "OCHK")) bad("object header continuation");
            if (len < 8) bad("object header continuation length");
            blocks.push_back({off + 4, off + len - 4});
          } else {
            out.push_back({type, d, size});
          }
          q = d + size;
        }
      }
    } else if (buf_[a] == 1) {
      const uint64_t nmsg = le(a + 2, 2), size = le(a + 8, 4);
      std::vector<std::pair<uint64_t, uint64_t>> blocks{{a + 16, a + 16 + size}};
      uint64_t seen = 0;
      for (size_t b = 0; b < blocks.size() && seen < nmsg; ++b) {
        if (b >= kMaxBlocks) bad("object header: too many continuation blocks (cycle?)");
        uint64_t q = blocks[b].first;
        while (q + 8 <= blocks[b].second && seen < nmsg) {
          const int type = (int)le(q, 2);
          const uint64_t sz = le(q + 2, 2);
          const uint64_t d = q + 8;
          need(d, sz);
          ++seen;
          if (type == 0x10)
            blocks.push_back({abs_(le(d, so_)), abs_(le(d, so_)) + le(d + so_, sl_)});
          else
            out.push_back({type, d, sz});
          q = d + sz;
        }
      }
    } else {
      bad("object header version");
    }
    return out;
  }

  // ---- root group -----------------------------------------------------------
  void read_group(uint64_t addr) {
    bool any = false;
    for (Msg const& m : messages(addr)) {
      if (m.type == 0x11) {  // symbol table: v1 B-tree of SNODs + local heap of names
        any = true;
        const uint64_t heap = abs_(le(m.at + so_, so_));
        if (!sig(heap, "HEAP")) bad("local heap");
        const uint64_t names = abs_(le(heap + 8 + 2 * sl_, so_));
        walk_group_btree(abs_(le(m.at, so_)), names);
      } else if (m.type == 0x06) {
        any = true;
        link(m.at);
      } else if (m.type == 0x02) {  // link info: dense storage when the heap exists
        any = true;
        const int flags = buf_[m.at + 1];
        uint64_t p = m.at + 2 + ((flags & 1) ? 8 : 0);
        const uint64_t fheap = le(p, so_), bt = le(p + so_, so_);
        if (!undef(fheap)) dense_links(abs_(fheap), abs_(bt));
      }
    }
    if (!any) bad("root object is not a group");
  }

  void walk_group_btree(uint64_t node, uint64_t names, int depth = 0) {
    if (depth > kMaxDepth) bad("group B-tree deeper than " + std::to_string(kMaxDepth));
    if (!sig(node, "TREE")) bad("group B-tree node");
    const int level = buf_[node + 5];
    const uint64_t n = le(node + 6, 2);
    uint64_t p = node + 8 + 2 * so_ + sl_;  // first child (after key 0)
    for (uint64_t i = 0; i < n; ++i, p += so_ + sl_) {
      const uint64_t child = abs_(le(p, so_));
      if (level > 0) {
        walk_group_btree(child, names, depth + 1);
        continue;
      }
      if (!sig(child, "SNOD")) bad("symbol table node");
      const uint64_t ns = le(child + 6, 2);
      for (uint64_t e = 0; e < ns; ++e) {
        const uint64_t ent = child + 8 + e * (2 * so_ + 24);
        const uint64_t noff = le(ent, so_), oh = le(ent + so_, so_);
        links_[cstr(names + noff)] = oh;
      }
    }
  }

  std::string cstr(uint64_t at) const {
    need(at, 1);
    const uint8_t* s = &buf_[at];
    const size_t n = strnlen(reinterpret_cast<const char*>(s), buf_.size() - at);
    return std::string(reinterpret_cast<const char*>(s), n);
  }

  // link message at `at`; returns its encoded length
  uint64_t link(uint64_t at) {
    const int flags = buf_.at(at + 1);
    uint64_t p = at + 2;
    int ltype = 0;
    if (flags & 0x08) ltype = buf_.at(p++);
    if (flags & 0x04) p += 8;
    if (flags & 0x10) p += 1;
    const int w = 1 << (flags & 3);
    const uint64_t nlen = le(p, w);
    p += w;
    need(p, nlen);
    std::string name(reinterpret_cast<const char*>(&buf_[p]), (size_t)nlen);
    p += nlen;
    if (ltype == 0) {
      links_[name] = le(p, so_);
      p += so_;
    } else {
      p += 2 + le(p, 2);  // soft / external links are not followed
    }
    return p - at;
  }

  // fractal heap + v2 B-tree (name index, record type 5: hash, heap ID)
  struct Heap {
    uint64_t hdr = 0;
    int id_len = 0, filt_len = 0, width = 0, max_heap_bits = 0, off_bytes = 0, len_bytes = 0;
    uint64_t start = 0, max_direct = 0, root = 0;
    int rows = 0;
    bool checksum_direct = false;
  };

  Heap heap_header(uint64_t h) const {
    if (!sig(h, "FRHP")) bad("fractal heap header");
    Heap H;
    H.hdr = h;
    uint64_t p = h + 5;
    H.id_len = (int)le(p, 2);
    H.filt_len = (int)le(p + 2, 2);
    const int flags = buf_.at(p + 4);
    H.checksum_direct = (flags & 0x02) != 0;
    const uint64_t max_obj = le(p + 5, 4);
    p += 9 + sl_ + so_ + sl_ + so_ + 8 * sl_;  // ... through the tiny-object counts
    H.width = (int)le(p, 2);
    H.start = le(p + 2, sl_);
    H.max_direct = le(p + 2 + sl_, sl_);
    H.max_heap_bits = (int)le(p + 2 + 2 * sl_, 2);
    p += 2 + 2 * sl_ + 2 + 2;  // + starting rows
    H.root = le(p, so_);
    H.rows = (int)le(p + so_, 2);
    H.off_bytes = (H.max_heap_bits + 7) / 8;
    const uint64_t lim = std::min<uint64_t>(H.max_direct, max_obj);
    int bits = 0;
    while (bits < 64 && (lim >> bits) != 0) ++bits;
    H.len_bytes = (bits + 7) / 8;
    if (1 + H.off_bytes + H.len_bytes != H.id_len) H.len_bytes = H.id_len - 1 - H.off_bytes;
    return H;
  }

  // file offset of heap offset `off` (managed objects)
  uint64_t heap_locate(Heap const& H, uint64_t off) const {
    if (H.rows == 0) return abs_(H.root) + off;  // root direct block at heap offset 0
    const uint64_t ib = abs_(H.root);
    if (!sig(ib, "FHIB")) bad("fractal heap indirect block");
    uint64_t p = ib + 5 + so_ + H.off_bytes;
    int lg_start = 0, lg_max = 0;
    while ((1ull << lg_start) < H.start) ++lg_start;
    while ((1ull << lg_max) < H.max_direct) ++lg_max;
    const int direct_rows = std::min(H.rows, lg_max - lg_start + 2);
    const int entry = so_ + (H.filt_len > 0 ? sl_ + 4 : 0);
    uint64_t boff = 0;
    for (int r = 0; r < direct_rows; ++r) {
      const uint64_t bsz = r < 2 ? H.start : H.start << (r - 1);
      for (int c = 0; c < H.width; ++c, boff += bsz, p += entry) {
        if (off >= boff && off < boff + bsz) {
          const uint64_t a = le(p, so_);
          if (undef(a)) bad("fractal heap: object in an unallocated block");
          return abs_(a) + (off - boff);
        }
      }
    }
    bad("fractal heap: nested indirect blocks are not supported");
  }

  // bytes needed to encode n (H5VM_limit_enc_size)
  static int enc_size(uint64_t n) {
    int lg = 0;
    while (lg < 63 && (n >> (lg + 1)) != 0) ++lg;
    return lg / 8 + 1;
  }

  void dense_links(uint64_t fheap, uint64_t bthd) {
    const Heap H = heap_header(fheap);
    if (!sig(bthd, "BTHD")) bad("v2 B-tree header");
    const uint64_t node_size = le(bthd + 6, 4);
    const int rec = (int)le(bthd + 10, 2);
    const int depth = (int)le(bthd + 12, 2);
    const uint64_t root = abs_(le(bthd + 16, so_));
    const uint64_t root_n = le(bthd + 16 + so_, 2);
    if (rec <= 0 || node_size <= 10 + (uint64_t)rec) bad("v2 B-tree record / node size");
    if (depth > kMaxDepth) bad("v2 B-tree deeper than " + std::to_string(kMaxDepth));
    // per-depth record counts and their encoded sizes (H5B2__hdr_init)
    std::vector<uint64_t> max_nrec(depth + 1), cum(depth + 1);
    std::vector<int> cum_size(depth + 1, 0);
    max_nrec[0] = (node_size - 10) / rec;
    cum[0] = max_nrec[0];
    const int max_nrec_size = enc_size(max_nrec[0]);
    for (int d = 1; d <= depth; ++d) {
      const int ptr = so_ + max_nrec_size + (d > 1 ? cum_size[d - 1] : 0);
      max_nrec[d] = (node_size - 10 - ptr) / (rec + ptr);
      cum[d] = (max_nrec[d] + 1) * cum[d - 1] + max_nrec[d];
      cum_size[d] = enc_size(cum[d]);
    }
    std::function<void(uint64_t, int, uint64_t)> walk = [&](uint64_t node, int d, uint64_t n) {
      const bool leaf = d == 0;
      if (!sig(node, leaf ? "BTLF" : "BTIN")) bad("v2 B-tree node");
      const uint64_t recs = node + 6;
      for (uint64_t i = 0; i < n; ++i) heap_link(H, recs + i * rec + 4);
      if (leaf) return;
      uint64_t p = recs + n * rec;
      for (uint64_t i = 0; i <= n; ++i) {
        const uint64_t child = abs_(le(p, so_));
        const uint64_t cn = le(p + so_, max_nrec_size);
        p += so_ + max_nrec_size + (d > 1 ? cum_size[d - 1] : 0);
        walk(child, d - 1, cn);
      }
    };
    if (!undef(le(bthd + 16, so_))) walk(root, depth, root_n);
  }

  void heap_link(Heap const& H, uint64_t id) {
    const int type = (buf_.at(id) >> 4) & 3;
    if (type == 0) {
      const uint64_t off = le(id + 1, H.off_bytes);
      link(heap_locate(H, off));
    } else if (type == 2) {  // tiny object inside the ID (normal form)
      link(id + 1);
    } else {
      bad("fractal heap: huge link objects are not supported");
    }
  }

  uint64_t lookup(std::string const& name) const {
    auto it = links_.find(name);
    if (it == links_.end())
      throw std::runtime_error(path_ + ": NetCDF: Variable not found (" + name + ")");
    return it->second;
  }

  // ---- datasets ---------------------------------------------------------------
  Dataset dataset(uint64_t addr) const {
    Dataset d;
    bool space = false;
    for (Msg const& m : messages(addr)) {
      const uint64_t a = m.at;
      switch (m.type) {
        case 0x01: {  // dataspace
          const int v = buf_.at(a), rank = buf_.at(a + 1);
          const uint64_t p = a + (v == 1 ? 8 : 4);
          for (int k = 0; k < rank; ++k) d.dims.push_back(le(p + k * sl_, sl_));
          space = true;
          break;
        }
        case 0x03: {  // datatype
          d.tclass = buf_.at(a) & 0x0F;
          const int bits = buf_.at(a + 1);
          d.big = (bits & 1) != 0;
          d.sign = (bits & 8) != 0;
          d.tsize = (int)le(a + 4, 4);
          break;
        }
        case 0x05: {  // fill value (versions 2, 3)
          const int v = buf_.at(a);
          if (v == 2 && buf_.at(a + 3)) {
            const uint64_t n = le(a + 4, 4);
            need(a + 8, n);
            d.fill.assign(&buf_[a + 8], &buf_[a + 8] + n);
          } else if (v == 3 && (buf_.at(a + 1) & 0x20)) {
            const uint64_t n = le(a + 2, 4);
            need(a + 6, n);
            d.fill.assign(&buf_[a + 6], &buf_[a + 6] + n);
          }
          break;
        }
        case 0x08: layout(d, a); break;
        case 0x0B: filters(d, a); break;
        default: break;
      }
    }
    if (!space || d.tclass < 0 || d.layout < 0) bad("object is not a dataset");
    if (d.tclass != 0 && d.tclass != 1) bad("only integer and floating-point variables are numeric");
    if (d.tsize != 1 && d.tsize != 2 && d.tsize != 4 && d.tsize != 8) bad("datatype size");
    if (d.tclass == 1 && d.tsize != 4 && d.tsize != 8) bad("float size");
    return d;
  }

  void layout(Dataset& d, uint64_t a) const {
    const int v = buf_.at(a);
    d.layout_version = v;
    if (v < 3) bad("data layout version " + std::to_string(v));
    d.layout = buf_.at(a + 1);
    uint64_t p = a + 2;
    if (d.layout == 0) {
      d.size = le(p, 2);
      d.compact_at = (size_t)(p + 2);
    } else if (d.layout == 1) {
      d.addr = le(p, so_);
      d.size = le(p + so_, sl_);
    } else if (d.layout == 2 && v == 3) {
      const int rank = buf_.at(p);
      d.addr = le(p + 1, so_);
      p += 1 + so_;
      for (int k = 0; k < rank - 1; ++k) d.chunk.push_back(le(p + 4 * k, 4));
    } else if (d.layout == 2 && v == 4) {
      const int flags = buf_.at(p), rank = buf_.at(p + 1), w = buf_.at(p + 2);
      p += 3;
      for (int k = 0; k < rank - 1; ++k) d.chunk.push_back(le(p + k * w, w));
      p += (uint64_t)rank * w;
      d.index_type = buf_.at(p++);
      if (d.index_type == 1) {
        if (flags & 0x02) {
          d.single_filtered = true;
          d.single_size = le(p, sl_);
          d.single_mask = (uint32_t)le(p + sl_, 4);
          p += sl_ + 4;
        }
      } else if (d.index_type == 3) {
        p += 1;  // page bits
      } else if (d.index_type != 2) {
        bad("chunk index type " + std::to_string(d.index_type) +
            " (extensible array / v2 B-tree) is not supported");
      }
      d.addr = le(p, so_);
    } else {
      bad("data layout class");
    }
  }

  void filters(Dataset& d, uint64_t a) const {
    const int v = buf_.at(a), n = buf_.at(a + 1);
    uint64_t p = a + (v == 1 ? 8 : 2);
    for (int f = 0; f < n; ++f) {
      const int id = (int)le(p, 2);
      uint64_t nlen = 0;
      p += 2;
      if (v == 1 || id >= 256) {
        nlen = le(p, 2);
        p += 2;
      }
      p += 2;  // flags
      const int nval = (int)le(p, 2);
      p += 2;
      if (v == 1) nlen = (nlen + 7) & ~7ull;
      p += nlen;
      std::vector<uint32_t> cd;
      for (int i = 0; i < nval; ++i) cd.push_back((uint32_t)le(p + 4 * i, 4));
      p += 4ull * nval;
      if (v == 1 && (nval & 1)) p += 4;
      d.filters.push_back({id, cd});
    }
  }

  std::vector<uint8_t> unfilter(Dataset const& d, std::vector<uint8_t> data, uint32_t mask,
                                size_t want) const {
    for (int f = (int)d.filters.size() - 1; f >= 0; --f) {
      if (mask & (1u << f)) continue;
      const int id = d.filters[f].first;
      if (id == 1) {  // deflate
        std::vector<uint8_t> out(want);
        uLongf n = (uLongf)want;
        if (uncompress(out.data(), &n, data.data(), (uLong)data.size()) != Z_OK || n != want)
          bad("deflate: corrupt chunk");
        data.swap(out);
      } else if (id == 2) {  // shuffle
        const size_t es = d.filters[f].second.empty() ? d.tsize : d.filters[f].second[0];
        if (es == 0) bad("shuffle: element size 0");
        const size_t ne = data.size() / es;
        std::vector<uint8_t> out(data.size());
        for (size_t b = 0; b < es; ++b)
          for (size_t e = 0; e < ne; ++e) out[e * es + b] = data[b * ne + e];
        std::copy(data.begin() + ne * es, data.end(), out.begin() + ne * es);
        data.swap(out);
      } else if (id == 3) {  // fletcher32: drop the trailing checksum
        if (data.size() < 4) bad("fletcher32: short chunk");
        data.resize(data.size() - 4);
      } else {
        bad("filter " + std::to_string(id) + " is not supported");
      }
    }
    if (data.size() < want) bad("chunk shorter than its extent");
    return data;
  }

  std::vector<uint8_t> read_raw(Dataset const& d) const {
    uint64_t n = 1;
    for (uint64_t x : d.dims) n *= x;
    const size_t bytes = (size_t)(n * d.tsize);
    std::vector<uint8_t> out(bytes);
    if (d.layout == 0) {
      need(d.compact_at, bytes);
      std::memcpy(out.data(), &buf_[d.compact_at], bytes);
      return out;
    }
    if (d.layout == 1) {
      if (undef(d.addr)) return filled(d, bytes);
      need(abs_(d.addr), bytes);
      std::memcpy(out.data(), &buf_[abs_(d.addr)], bytes);
      return out;
    }
    // chunked: start from the fill value, then place every stored chunk
    out = filled(d, bytes);
    const int rank = (int)d.dims.size();
    size_t cbytes = d.tsize;
    for (uint64_t c : d.chunk) cbytes *= c;
    auto place = [&](std::vector<uint64_t> const& origin, uint64_t addr, uint64_t size,
                     uint32_t mask) {
      need(abs_(addr), size);
      std::vector<uint8_t> raw(&buf_[abs_(addr)], &buf_[abs_(addr)] + size);
      std::vector<uint8_t> c = d.filters.empty() ? raw : unfilter(d, raw, mask, cbytes);
      if (c.size() < cbytes) bad("chunk shorter than its extent");
      // copy the chunk's rows that fall inside the dataset (edge chunks overhang)
      std::vector<uint64_t> idx(rank, 0);
      const uint64_t inner = d.chunk[rank - 1];
      for (;;) {
        uint64_t src = 0, dst = 0;
        bool inside = true;
        for (int k = 0; k < rank; ++k) {
          const uint64_t g = origin[k] + idx[k];
          if (g >= d.dims[k]) inside = false;
          src = src * d.chunk[k] + idx[k];
          dst = dst * d.dims[k] + g;
        }
        if (inside) {
          const uint64_t cnt = std::min<uint64_t>(inner, d.dims[rank - 1] - origin[rank - 1]);
          std::memcpy(&out[dst * d.tsize], &c[src * d.tsize], cnt * d.tsize);
        }
        int k = rank - 2;
        for (; k >= 0; --k) {
          if (++idx[k] < d.chunk[k]) break;
          idx[k] = 0;
        }
        if (k < 0) break;
      }
    };
    if (rank == 0) bad("chunked scalar");
    if ((int)d.chunk.size() != rank) bad("chunk rank differs from the dataspace rank");
    for (uint64_t cdim : d.chunk)
      if (cdim == 0) bad("chunk dimension 0");
    std::vector<uint64_t> grid(rank);
    uint64_t nchunks = 1;
    for (int k = 0; k < rank; ++k) {
      grid[k] = (d.dims[k] + d.chunk[k] - 1) / d.chunk[k];
      nchunks *= grid[k];
    }
    auto origin_of = [&](uint64_t lin) {
      std::vector<uint64_t> o(rank);
      for (int k = rank - 1; k >= 0; --k) {
        o[k] = (lin % grid[k]) * d.chunk[k];
        lin /= grid[k];
      }
      return o;
    };
    if (undef(d.addr)) return out;
    if (d.layout_version == 3) {
      btree_chunks(d, abs_(d.addr), rank, place);
    } else if (d.index_type == 1) {
      place(std::vector<uint64_t>(rank, 0), d.addr, d.single_filtered ? d.single_size : cbytes,
            d.single_mask);
    } else if (d.index_type == 2) {
      for (uint64_t i = 0; i < nchunks; ++i) place(origin_of(i), d.addr + i * cbytes, cbytes, 0);
    } else {  // fixed array
      const uint64_t h = abs_(d.addr);
      if (!sig(h, "FAHD")) bad("fixed array header");
      const int client = buf_.at(h + 5), esz = buf_.at(h + 6), pbits = buf_.at(h + 7);
      const uint64_t nent = le(h + 8, sl_);
      const uint64_t db = abs_(le(h + 8 + sl_, so_));
      if (nent > (1ull << pbits)) bad("paged fixed array");
      if (!sig(db, "FADB")) bad("fixed array data block");
      uint64_t p = db + 6 + so_;
      for (uint64_t i = 0; i < nent && i < nchunks; ++i, p += esz) {
        const uint64_t addr = le(p, so_);
        if (undef(addr)) continue;
        if (client == 0) {
          place(origin_of(i), addr, cbytes, 0);
        } else {
          const int w = esz - so_ - 4;
          place(origin_of(i), addr, le(p + so_, w), (uint32_t)le(p + so_ + w, 4));
        }
      }
    }
    return out;
  }

  template <class Place>
  void btree_chunks(Dataset const& d, uint64_t node, int rank, Place& place, int depth = 0) const {
    if (depth > kMaxDepth) bad("chunk B-tree deeper than " + std::to_string(kMaxDepth));
    if (!sig(node, "TREE")) bad("chunk B-tree node");
    if (buf_[node + 4] != 1) bad("chunk B-tree type");
    const int level = buf_[node + 5];
    const uint64_t n = le(node + 6, 2);
    const uint64_t key = 8 + 8ull * (rank + 1);
    uint64_t p = node + 8 + 2 * so_;
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t size = le(p, 4);
      const uint32_t mask = (uint32_t)le(p + 4, 4);
      std::vector<uint64_t> origin(rank);
      for (int k = 0; k < rank; ++k) {
        origin[k] = le(p + 8 + 8ull * k, 8);
        if (level == 0 && origin[k] % d.chunk[k]) bad("chunk origin off the chunk grid");
      }
      const uint64_t child = le(p + key, so_);
      if (level > 0)
        btree_chunks(d, abs_(child), rank, place, depth + 1);
      else
        place(origin, child, size, mask);
      p += key + so_;
    }
  }

  std::vector<uint8_t> filled(Dataset const& d, size_t bytes) const {
    std::vector<uint8_t> out(bytes, 0);
    if ((int)d.fill.size() == d.tsize)
      for (size_t i = 0; i + d.tsize <= bytes; i += d.tsize)
        std::memcpy(&out[i], d.fill.data(), d.tsize);
    return out;
  }

  static double convert(Dataset const& d, const uint8_t* p) {
    uint64_t x = 0;
    for (int i = 0; i < d.tsize; ++i) {
      const int b = d.big ? i : d.tsize - 1 - i;
      x = (x << 8) | p[b];
    }
    if (d.tclass == 1) {
      if (d.tsize == 8) {
        double v;
        std::memcpy(&v, &x, 8);
        return v;
      }
      const uint32_t u = (uint32_t)x;
      float v;
      std::memcpy(&v, &u, 4);
      return v;
    }
    if (!d.sign) return (double)x;
    const int sh = 64 - 8 * d.tsize;
    return (double)((int64_t)(x << sh) >> sh);
  }
};

}  // namespace harp_amd
