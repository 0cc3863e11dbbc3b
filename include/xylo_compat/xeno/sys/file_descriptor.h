// xeno/sys/file_descriptor.h (xylo-hip drop-in layer): the read-only file
// mapping deep_agent.cc uses to load `weights.NN` (xeno/sys/file_descriptor.h:
// 270-316).  Pages are mapped private, so writes through span() stay local.
#ifndef XYLO_HIP_COMPAT_XENO_SYS_FILE_DESCRIPTOR_H_
#define XYLO_HIP_COMPAT_XENO_SYS_FILE_DESCRIPTOR_H_

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstddef>
#include <filesystem>
#include <span>
#include <utility>

#include <xeno/exception.h>

namespace xeno {
namespace sys {

template <typename T> class mmap {
 public:
  mmap() = default;
  explicit mmap(const std::filesystem::path &p, std::size_t size = -1) {
    const int fd = ::open(p.c_str(), O_RDONLY);
    if (fd < 0) throw xeno::error("mmap: cannot open " + p.string());
    struct stat st {};
    ::fstat(fd, &st);
    if (size == std::size_t(-1)) size = std::size_t(st.st_size) / sizeof(T);
    void *ptr = size ? ::mmap(nullptr, size * sizeof(T), PROT_READ | PROT_WRITE,
                              MAP_PRIVATE, fd, 0)
                     : nullptr;
    ::close(fd);
    if (ptr == MAP_FAILED) throw xeno::error("mmap failed");
    data_ = std::span<T>(static_cast<T *>(ptr), size);
  }
  ~mmap() {
    if (!data_.empty()) ::munmap(data_.data(), data_.size_bytes());
  }
  mmap(const mmap &) = delete;
  void operator=(const mmap &) = delete;
  mmap(mmap &&o) noexcept : data_(std::exchange(o.data_, {})) {}
  mmap &operator=(mmap &&o) noexcept {
    std::swap(data_, o.data_);
    return *this;
  }

  std::span<T> span() const { return data_; }

 private:
  std::span<T> data_;
};

}  // namespace sys
}  // namespace xeno

#endif  // XYLO_HIP_COMPAT_XENO_SYS_FILE_DESCRIPTOR_H_
