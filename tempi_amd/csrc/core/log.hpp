// tempi_amd/csrc/core/log.hpp -- run-time log levels (the reference fixes the
// level at compile time: /root/reference/include/logging.hpp:29-77; here
// TEMPI_LOG_LEVEL=SPEW|DEBUG|INFO|WARN|ERROR|FATAL picks it at MPI_Init).
#pragma once

#include <cstdio>
#include <cstdlib>
#include <sstream>

namespace tempi {

enum class Level { SPEW = 0, DEBUG, INFO, WARN, ERROR, FATAL };

extern Level logLevel;
extern int logRank;

void log_line(Level l, const std::string &msg);
[[noreturn]] void fatal(const std::string &msg);

} // namespace tempi

#define TEMPI_LOG(lvl, expr)                                                   \
  do {                                                                         \
    if (int(tempi::Level::lvl) >= int(tempi::logLevel)) {                      \
      std::ostringstream tempi_ss_;                                            \
      tempi_ss_ << expr;                                                       \
      tempi::log_line(tempi::Level::lvl, tempi_ss_.str());                     \
    }                                                                          \
  } while (0)

#define LOG_SPEW(expr) TEMPI_LOG(SPEW, expr)
#define LOG_DEBUG(expr) TEMPI_LOG(DEBUG, expr)
#define LOG_INFO(expr) TEMPI_LOG(INFO, expr)
#define LOG_WARN(expr) TEMPI_LOG(WARN, expr)
#define LOG_ERROR(expr) TEMPI_LOG(ERROR, expr)
#define LOG_FATAL(expr)                                                        \
  do {                                                                         \
    std::ostringstream tempi_ss_;                                              \
    tempi_ss_ << expr;                                                         \
    tempi::fatal(tempi_ss_.str());                                             \
  } while (0)
