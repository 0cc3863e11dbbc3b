// xeno/exception.h (xylo-hip drop-in layer): the reference's error type
// (xeno/exception.h:10-22).  The C ABI never throws; the C++ layer turns a
// non-zero xh status into this exception, keeping the reference convention.
#ifndef XYLO_HIP_COMPAT_XENO_EXCEPTION_H_
#define XYLO_HIP_COMPAT_XENO_EXCEPTION_H_

#include <source_location>
#include <stdexcept>
#include <string>
#include <string_view>

namespace xeno {

class error : public std::runtime_error {
 public:
  error(std::string_view message,
        std::source_location location = std::source_location::current())
      : std::runtime_error(std::string(message)), location_(location) {}

  std::source_location location() const { return location_; }

 private:
  std::source_location location_;
};

}  // namespace xeno

#endif  // XYLO_HIP_COMPAT_XENO_EXCEPTION_H_
