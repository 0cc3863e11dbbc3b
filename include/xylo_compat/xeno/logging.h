// xeno/logging.h (xylo-hip drop-in layer): `lg() << ...` writes one line to
// stderr when the temporary dies, like the reference's logstream
// (xeno/logging.h:43-97): "<local time> I <file>:<line>:\t<message>".
#ifndef XYLO_HIP_COMPAT_XENO_LOGGING_H_
#define XYLO_HIP_COMPAT_XENO_LOGGING_H_

#include <ctime>
#include <iostream>
#include <source_location>
#include <sstream>
#include <string>

namespace xeno {
namespace logging {

class logstream : public std::ostringstream {
 public:
  enum level { info, warning, error, fatal };

  explicit logstream(level l = info,
                     std::source_location loc = std::source_location::current())
      : level_(l), loc_(loc) {}
  logstream(std::source_location loc) : level_(info), loc_(loc) {}
  ~logstream() override {
    char ts[32];
    const std::time_t now = std::time(nullptr);
    std::strftime(ts, sizeof ts, "%Y-%m-%d %H:%M:%S", std::localtime(&now));
    std::string file = loc_.file_name();
    const auto slash = file.find_last_of('/');
    if (slash != std::string::npos) file = file.substr(slash + 1);
    std::ostringstream line;
    line << ts << ' ' << "IWEF"[level_] << ' ' << file << ':' << loc_.line()
         << ":\t" << str() << '\n';
    std::cerr << line.str();
  }

 private:
  level level_;
  std::source_location loc_;
};

}  // namespace logging
using log = logging::logstream;
}  // namespace xeno

using lg = xeno::log;

#endif  // XYLO_HIP_COMPAT_XENO_LOGGING_H_
