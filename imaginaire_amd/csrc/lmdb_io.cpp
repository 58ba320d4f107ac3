// Native LMDB (data.mdb) reader + bulk writer for the dataset pipeline.
//
// The reference reads its datasets through the `lmdb` Python binding
// (reference datasets/lmdb.py:17-79, utils/lmdb.py:43-75). That package is
// not part of this stack, so the on-disk format is implemented here directly:
//
//   * Reader: mmaps <root>/data.mdb read-only, picks the newer of the two
//     meta pages and answers get(key) by walking the main B+tree (branch
//     pages -> leaf page -> inline value or overflow pages). No locks, no
//     copies: values are returned as views of the mapping. Thread-safe and
//     fork-safe (each DataLoader worker shares the page cache).
//   * Writer: builds a complete, valid single-transaction LMDB file from
//     sorted (key, value) pairs in one pass — leaf pages filled bottom-up,
//     values larger than the node limit spilled into overflow pages, branch
//     levels built until a single root remains, then both meta pages.
//
// Layout constants follow LMDB's on-disk format for 64-bit builds
// (page header 16 B, node header 8 B, meta record at offset 16 of pages
// 0/1, MDB_db 48 B, default 4 KiB pages).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#ifndef IAMD_LMDB_NO_PYTHON
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;
#endif

namespace iamd {
namespace lmdb {

constexpr uint32_t kMagic = 0xBEEFC0DE;
constexpr uint32_t kVersion = 1;
constexpr size_t kPageHdr = 16;
constexpr size_t kNodeHdr = 8;
constexpr uint16_t P_BRANCH = 0x01, P_LEAF = 0x02, P_OVERFLOW = 0x04, P_META = 0x08,
                   P_LEAF2 = 0x20;
constexpr uint16_t F_BIGDATA = 0x01, F_SUBDATA = 0x02, F_DUPDATA = 0x04;
constexpr uint64_t kInvalidPage = ~0ULL;

#pragma pack(push, 1)
struct DbRec {  // MDB_db
  uint32_t pad;
  uint16_t flags;
  uint16_t depth;
  uint64_t branch_pages;
  uint64_t leaf_pages;
  uint64_t overflow_pages;
  uint64_t entries;
  uint64_t root;
};
struct MetaRec {  // MDB_meta
  uint32_t magic;
  uint32_t version;
  uint64_t address;
  uint64_t mapsize;
  DbRec dbs[2];
  uint64_t last_pg;
  uint64_t txnid;
};
struct PageHdr {
  uint64_t pgno;
  uint16_t pad;
  uint16_t flags;
  uint16_t lower;
  uint16_t upper;
};
struct NodeHdr {
  uint16_t lo;
  uint16_t hi;
  uint16_t flags;
  uint16_t ksize;
};
#pragma pack(pop)
static_assert(sizeof(DbRec) == 48, "MDB_db layout");
static_assert(sizeof(MetaRec) == 136, "MDB_meta layout");
static_assert(sizeof(PageHdr) == kPageHdr, "page header layout");
static_assert(sizeof(NodeHdr) == kNodeHdr, "node header layout");

inline int key_cmp(const char* a, size_t na, const char* b, size_t nb) {
  int c = std::memcmp(a, b, std::min(na, nb));
  if (c) return c;
  return na < nb ? -1 : (na > nb ? 1 : 0);
}

class Reader {
 public:
  explicit Reader(const std::string& root) {
    std::string path = root;
    struct stat st;
    if (::stat(path.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) path += "/data.mdb";
    fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd_ < 0) throw std::runtime_error("lmdb: cannot open " + path);
    if (::fstat(fd_, &st) != 0) throw std::runtime_error("lmdb: stat failed " + path);
    size_ = static_cast<size_t>(st.st_size);
    if (size_ < 2 * kPageHdr + 2 * sizeof(MetaRec))
      throw std::runtime_error("lmdb: file too small " + path);
    base_ = static_cast<const char*>(::mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0));
    if (base_ == MAP_FAILED) throw std::runtime_error("lmdb: mmap failed " + path);
    ::madvise(const_cast<char*>(base_), size_, MADV_RANDOM);
    const MetaRec* m0 = meta_at(0, 0);
    psize_ = m0->dbs[0].pad ? m0->dbs[0].pad : 4096;
    if (psize_ < 512 || psize_ > (1u << 16) || (psize_ & (psize_ - 1)))
      throw std::runtime_error("lmdb: bad page size in " + path);
    const MetaRec* m1 = meta_at(1, psize_);
    const MetaRec* m = m0;
    if (m1 && m1->magic == kMagic && (m0->magic != kMagic || m1->txnid > m0->txnid)) m = m1;
    if (m->magic != kMagic) throw std::runtime_error("lmdb: bad magic in " + path);
    if (m->version != kVersion) throw std::runtime_error("lmdb: unsupported version");
    main_ = m->dbs[1];
    if (main_.flags & 0x04 /*MDB_DUPSORT*/)
      throw std::runtime_error("lmdb: DUPSORT databases are not supported");
  }
  ~Reader() {
    if (base_ && base_ != MAP_FAILED) ::munmap(const_cast<char*>(base_), size_);
    if (fd_ >= 0) ::close(fd_);
  }
  Reader(const Reader&) = delete;
  Reader& operator=(const Reader&) = delete;

  uint64_t entries() const { return main_.entries; }
  uint32_t page_size() const { return psize_; }

  // Returns (pointer, size) of the value, or (nullptr, 0) if absent.
  std::pair<const char*, size_t> get(const std::string& key) const {
    if (main_.root == kInvalidPage) return {nullptr, 0};
    uint64_t pg = main_.root;
    for (int guard = 0; guard < 64; ++guard) {
      const char* p = page(pg);
      const PageHdr* h = reinterpret_cast<const PageHdr*>(p);
      const int n = num_keys(h);
      if (h->flags & P_BRANCH) {
        if (n < 1) throw std::runtime_error("lmdb: empty branch page");
        // last node whose key <= search key (node 0 = -inf)
        int lo = 1, hi = n - 1, idx = 0;
        while (lo <= hi) {
          int mid = (lo + hi) / 2;
          const NodeHdr* nd = node(p, mid);
          int c = key_cmp(key.data(), key.size(), node_key(nd), nd->ksize);
          if (c >= 0) {
            idx = mid;
            lo = mid + 1;
          } else {
            hi = mid - 1;
          }
        }
        const NodeHdr* nd = node(p, idx);
        pg = uint64_t(nd->lo) | (uint64_t(nd->hi) << 16) | (uint64_t(nd->flags) << 32);
        continue;
      }
      if (!(h->flags & P_LEAF) || (h->flags & P_LEAF2))
        throw std::runtime_error("lmdb: unexpected page type");
      int lo = 0, hi = n - 1;
      while (lo <= hi) {
        int mid = (lo + hi) / 2;
        const NodeHdr* nd = node(p, mid);
        int c = key_cmp(key.data(), key.size(), node_key(nd), nd->ksize);
        if (c == 0) return value_of(nd);
        if (c > 0) lo = mid + 1; else hi = mid - 1;
      }
      return {nullptr, 0};
    }
    throw std::runtime_error("lmdb: tree too deep (corrupt file?)");
  }

  // In-order traversal of all keys.
  std::vector<std::string> keys() const {
    std::vector<std::string> out;
    if (main_.root != kInvalidPage) walk(main_.root, out, 0);
    return out;
  }

 private:
  const MetaRec* meta_at(int idx, uint32_t psize) const {
    size_t off = (size_t)idx * psize + kPageHdr;
    if (off + sizeof(MetaRec) > size_) return nullptr;
    return reinterpret_cast<const MetaRec*>(base_ + off);
  }
  const char* page(uint64_t pg) const {
    if (pg >= size_ / psize_) throw std::runtime_error("lmdb: page out of range");
    return base_ + (size_t)pg * psize_;
  }
  // Every field read from the file is bounds-checked against the page before it is used:
  // a truncated or corrupted data.mdb raises instead of reading outside the mapping
  // (tests/native/lmdb_sanitize.cpp fuzzes this under ASan + UBSan).
  int num_keys(const PageHdr* h) const {
    if (h->lower < kPageHdr || h->lower > psize_ || (h->lower - kPageHdr) % 2)
      throw std::runtime_error("lmdb: corrupt page header");
    return (h->lower - kPageHdr) >> 1;
  }
  const NodeHdr* node(const char* p, int i) const {
    uint16_t off;
    std::memcpy(&off, p + kPageHdr + 2 * i, 2);
    // LMDB keeps nodes 2-byte aligned; an odd offset is corruption (and would make every
    // NodeHdr field access misaligned)
    if (off < kPageHdr || (off & 1) || (size_t)off + kNodeHdr > psize_)
      throw std::runtime_error("lmdb: corrupt node offset");
    const NodeHdr* nd = reinterpret_cast<const NodeHdr*>(p + off);
    if ((size_t)off + kNodeHdr + nd->ksize > psize_)
      throw std::runtime_error("lmdb: corrupt key size");
    return nd;
  }
  static const char* node_key(const NodeHdr* nd) {
    return reinterpret_cast<const char*>(nd) + kNodeHdr;
  }
  std::pair<const char*, size_t> value_of(const NodeHdr* nd) const {
    const size_t dsize = size_t(nd->lo) | (size_t(nd->hi) << 16);
    const char* d = node_key(nd) + nd->ksize;
    if (nd->flags & (F_SUBDATA | F_DUPDATA))
      throw std::runtime_error("lmdb: sub-databases are not supported");
    // node() checked the header and key against the page; the value must fit as well
    const size_t in_page = (size_t)(d - base_) % psize_;
    if (nd->flags & F_BIGDATA) {
      if (in_page + 8 > psize_) throw std::runtime_error("lmdb: corrupt overflow link");
      uint64_t opg;
      std::memcpy(&opg, d, 8);
      if (opg >= size_ / psize_ || dsize > size_ - (size_t)opg * psize_ - kPageHdr)
        throw std::runtime_error("lmdb: overflow out of range");
      return {page(opg) + kPageHdr, dsize};
    }
    if (in_page + dsize > psize_) throw std::runtime_error("lmdb: corrupt value size");
    return {d, dsize};
  }
  void walk(uint64_t pg, std::vector<std::string>& out, int depth) const {
    if (depth > 64) throw std::runtime_error("lmdb: tree too deep");
    const char* p = page(pg);
    const PageHdr* h = reinterpret_cast<const PageHdr*>(p);
    const int n = num_keys(h);
    for (int i = 0; i < n; ++i) {
      const NodeHdr* nd = node(p, i);
      if (h->flags & P_BRANCH) {
        walk(uint64_t(nd->lo) | (uint64_t(nd->hi) << 16) | (uint64_t(nd->flags) << 32), out,
             depth + 1);
      } else {
        out.emplace_back(node_key(nd), static_cast<size_t>(nd->ksize));
      }
    }
  }

  int fd_ = -1;
  size_t size_ = 0;
  const char* base_ = nullptr;
  uint32_t psize_ = 4096;
  DbRec main_{};
};

// ----------------------------------------------------------------- writer
class Writer {
 public:
  explicit Writer(uint32_t psize) : psize_(psize) {
    nodemax_ = ((psize_ - kPageHdr) / 2) & ~1u;  // MDB_MINKEYS = 2
    pages_.resize(2 * psize_, 0);               // meta pages 0 and 1
  }

  void build(std::vector<std::pair<std::string, std::string>>& kv) {
    std::sort(kv.begin(), kv.end(), [](const auto& a, const auto& b) {
      return key_cmp(a.first.data(), a.first.size(), b.first.data(), b.first.size()) < 0;
    });
    for (size_t i = 1; i < kv.size(); ++i)
      if (kv[i].first == kv[i - 1].first) throw std::runtime_error("lmdb: duplicate key");
    for (auto& e : kv)
      if (e.first.empty() || e.first.size() > 511)
        throw std::runtime_error("lmdb: key size must be 1..511 bytes");
    entries_ = kv.size();
    // ---- leaves (+ overflow pages for big values)
    struct Child { uint64_t pgno; std::string first_key; };
    std::vector<Child> level;
    start_page(P_LEAF);
    std::string first;
    bool empty = true;
    for (auto& e : kv) {
      const std::string& k = e.first;
      const std::string& v = e.second;
      bool big = kNodeHdr + k.size() + v.size() > nodemax_;
      size_t dsz = big ? 8 : v.size();
      size_t need = even(kNodeHdr + k.size() + dsz) + 2;
      if (!empty && need > free_space()) {
        level.push_back({cur_pgno_, first});
        finish_page();
        ++leaf_pages_;
        start_page(P_LEAF);
        empty = true;
      }
      uint64_t opg = 0;
      if (big) opg = write_overflow(v);  // appended after the current page is reserved
      add_node(k, big ? std::string(reinterpret_cast<const char*>(&opg), 8) : v, v.size(),
               big ? F_BIGDATA : 0, 0);
      if (empty) first = k;
      empty = false;
    }
    if (!empty) {
      level.push_back({cur_pgno_, first});
      finish_page();
      ++leaf_pages_;
    } else {
      abandon_page();
    }
    depth_ = level.empty() ? 0 : 1;
    // ---- branch levels
    while (level.size() > 1) {
      std::vector<Child> up;
      start_page(P_BRANCH);
      bool fresh = true;
      std::string pfirst;
      for (auto& c : level) {
        const std::string key = fresh ? std::string() : c.first_key;
        size_t need = even(kNodeHdr + key.size()) + 2;
        if (!fresh && need > free_space()) {
          up.push_back({cur_pgno_, pfirst});
          finish_page();
          ++branch_pages_;
          start_page(P_BRANCH);
          fresh = true;
        }
        add_node(fresh ? std::string() : c.first_key, std::string(), 0, 0, c.pgno);
        if (fresh) pfirst = c.first_key;
        fresh = false;
      }
      up.push_back({cur_pgno_, pfirst});
      finish_page();
      ++branch_pages_;
      level.swap(up);
      ++depth_;
    }
    root_ = level.empty() ? kInvalidPage : level[0].pgno;
    write_metas();
  }

  const std::vector<char>& data() const { return pages_; }

 private:
  static size_t even(size_t n) { return (n + 1) & ~size_t(1); }
  char* page_ptr(uint64_t pg) { return pages_.data() + pg * psize_; }
  size_t free_space() const { return upper_ - lower_; }

  void start_page(uint16_t flags) {
    cur_pgno_ = pages_.size() / psize_;
    pages_.resize(pages_.size() + psize_, 0);
    cur_flags_ = flags;
    lower_ = kPageHdr;
    upper_ = psize_;
  }
  void abandon_page() { pages_.resize(pages_.size() - psize_); }
  void finish_page() {
    PageHdr h{cur_pgno_, 0, cur_flags_, (uint16_t)lower_, (uint16_t)upper_};
    std::memcpy(page_ptr(cur_pgno_), &h, sizeof(h));
  }
  void add_node(const std::string& key, const std::string& data, size_t dsize_field,
                uint16_t flags, uint64_t child) {
    const size_t sz = even(kNodeHdr + key.size() + data.size());
    upper_ -= sz;
    char* p = page_ptr(cur_pgno_);
    NodeHdr nd{};
    if (cur_flags_ & P_BRANCH) {
      nd.lo = child & 0xffff;
      nd.hi = (child >> 16) & 0xffff;
      nd.flags = (child >> 32) & 0xffff;
    } else {
      nd.lo = dsize_field & 0xffff;
      nd.hi = (dsize_field >> 16) & 0xffff;
      nd.flags = flags;
    }
    nd.ksize = (uint16_t)key.size();
    std::memcpy(p + upper_, &nd, kNodeHdr);
    std::memcpy(p + upper_ + kNodeHdr, key.data(), key.size());
    std::memcpy(p + upper_ + kNodeHdr + key.size(), data.data(), data.size());
    uint16_t off = (uint16_t)upper_;
    std::memcpy(p + lower_, &off, 2);
    lower_ += 2;
  }
  uint64_t write_overflow(const std::string& v) {
    const size_t npages = (kPageHdr + v.size() + psize_ - 1) / psize_;
    const uint64_t pg = pages_.size() / psize_;
    pages_.resize(pages_.size() + npages * psize_, 0);
    char* p = page_ptr(pg);
    PageHdr h{pg, 0, P_OVERFLOW, 0, 0};
    uint32_t n32 = (uint32_t)npages;
    std::memcpy(p, &h, sizeof(h));
    std::memcpy(p + 12, &n32, 4);  // pb_pages overlays lower/upper
    std::memcpy(p + kPageHdr, v.data(), v.size());
    overflow_pages_ += npages;
    return pg;
  }
  void write_metas() {
    const uint64_t npages = pages_.size() / psize_;
    for (int i = 0; i < 2; ++i) {
      MetaRec m{};
      m.magic = kMagic;
      m.version = kVersion;
      m.address = 0;
      m.mapsize = std::max<uint64_t>(npages * psize_, 1ULL << 20);
      m.dbs[0].pad = psize_;
      m.dbs[0].root = kInvalidPage;
      m.dbs[1].depth = (uint16_t)depth_;
      m.dbs[1].branch_pages = branch_pages_;
      m.dbs[1].leaf_pages = leaf_pages_;
      m.dbs[1].overflow_pages = overflow_pages_;
      m.dbs[1].entries = entries_;
      m.dbs[1].root = root_;
      m.last_pg = npages - 1;
      m.txnid = (uint64_t)i;
      PageHdr h{(uint64_t)i, 0, P_META, 0, 0};
      std::memcpy(page_ptr(i), &h, sizeof(h));
      std::memcpy(page_ptr(i) + kPageHdr, &m, sizeof(m));
    }
  }

  uint32_t psize_;
  size_t nodemax_;
  std::vector<char> pages_;
  uint64_t cur_pgno_ = 0;
  uint16_t cur_flags_ = 0;
  size_t lower_ = 0, upper_ = 0;
  uint64_t entries_ = 0, leaf_pages_ = 0, branch_pages_ = 0, overflow_pages_ = 0;
  uint64_t root_ = kInvalidPage;
  int depth_ = 0;
};

void write_lmdb(const std::string& root, std::vector<std::pair<std::string, std::string>> kv,
                uint32_t page_size) {
  Writer w(page_size);
  w.build(kv);
  ::mkdir(root.c_str(), 0755);
  const std::string path = root + "/data.mdb";
  const std::string tmp = path + ".tmp";
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("lmdb: cannot create " + tmp);
  const auto& d = w.data();
  size_t done = 0;
  while (done < d.size()) {
    ssize_t r = ::write(fd, d.data() + done, d.size() - done);
    if (r <= 0) {
      ::close(fd);
      throw std::runtime_error("lmdb: write failed " + tmp);
    }
    done += (size_t)r;
  }
  ::fsync(fd);
  ::close(fd);
  if (::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("lmdb: rename failed");
}

}  // namespace lmdb

#ifndef IAMD_LMDB_NO_PYTHON
void register_lmdb(py::module_& m) {
  using lmdb::Reader;
  py::class_<Reader, std::shared_ptr<Reader>>(m, "LmdbReader")
      .def(py::init<const std::string&>(), py::arg("path"))
      .def("__len__", [](const Reader& r) { return r.entries(); })
      .def("page_size", &Reader::page_size)
      .def("get",
           [](const Reader& r, py::bytes key) -> py::object {
             auto v = r.get(std::string(key));
             if (!v.first) return py::none();
             return py::bytes(v.first, v.second);
           },
           py::arg("key"), "value bytes for key (None if absent)")
      .def("get_many",
           [](const Reader& r, const std::vector<std::string>& keys) {
             py::list out;
             for (const auto& k : keys) {
               auto v = r.get(k);
               if (v.first) out.append(py::bytes(v.first, v.second));
               else out.append(py::none());
             }
             return out;
           })
      .def("keys", [](const Reader& r) {
        py::list out;
        for (auto& k : r.keys()) out.append(py::bytes(k));
        return out;
      });
  m.def("lmdb_write",
        [](const std::string& root, const std::vector<std::pair<py::bytes, py::bytes>>& items,
           uint32_t page_size) {
          std::vector<std::pair<std::string, std::string>> kv;
          kv.reserve(items.size());
          for (auto& it : items) kv.emplace_back(std::string(it.first), std::string(it.second));
          py::gil_scoped_release nogil;
          lmdb::write_lmdb(root, std::move(kv), page_size);
        },
        py::arg("root"), py::arg("items"), py::arg("page_size") = 4096,
        "write a fresh LMDB environment (<root>/data.mdb) from (key, value) bytes pairs");
}

#endif  // IAMD_LMDB_NO_PYTHON

}  // namespace iamd
