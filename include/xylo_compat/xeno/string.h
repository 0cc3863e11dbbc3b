// xeno/string.h (xylo-hip drop-in layer): strcat / streamable / join, the
// formatting helpers the drivers and bin_packing.h use (xeno/string.h:39-134).
#ifndef XYLO_HIP_COMPAT_XENO_STRING_H_
#define XYLO_HIP_COMPAT_XENO_STRING_H_

#include <ranges>
#include <sstream>
#include <string>
#include <string_view>
#include <utility>

namespace xeno {
namespace string {

template <typename... Types> std::string strcat(Types... args) {
  std::ostringstream oss;
  (oss << ... << args);
  return oss.str();
}

template <typename T>
concept text = std::is_convertible_v<const T &, std::string_view>;

template <typename T1, typename T2>
std::string streamable(const std::pair<T1, T2> &p, std::string_view = ",") {
  return strcat('(', p.first, ',', p.second, ')');
}

template <typename T>
std::string streamable(const T &t, std::string_view sep = ",") {
  if constexpr (std::ranges::range<T> && !text<T>) {
    std::ostringstream oss;
    oss << '[';
    bool first = true;
    for (const auto &item : t) {
      if (!first) oss << sep;
      first = false;
      oss << streamable(item, sep);
    }
    oss << ']';
    return oss.str();
  } else {
    std::ostringstream oss;
    oss << t;
    return oss.str();
  }
}

template <std::ranges::range T> std::string join(T &&v, char sep = ',') {
  std::ostringstream oss;
  bool first = true;
  for (const auto &x : v) {
    if (!first) oss << sep;
    first = false;
    oss << x;
  }
  return oss.str();
}

}  // namespace string
}  // namespace xeno

#endif  // XYLO_HIP_COMPAT_XENO_STRING_H_
