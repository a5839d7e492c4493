// tempi_amd/csrc/core/env.cpp -- see env.hpp
#include "env.hpp"
#include "log.hpp"

#include <cstdlib>
#include <cstring>
#include <unistd.h>

namespace tempi {

Environment env;
Level logLevel = Level::WARN;
int logRank = -1;

static bool has(const char *name) { return std::getenv(name) != nullptr; }

void read_environment() {
  Environment e;
  e.noTempi = has("TEMPI_DISABLE");
  e.noPack = has("TEMPI_NO_PACK");
  e.noTypeCommit = has("TEMPI_NO_TYPE_COMMIT");
  e.faultPack = has("TEMPI_FAULT_PACK");

  if (has("TEMPI_ALLTOALLV_REMOTE_FIRST")) e.alltoallv = AlltoallvMethod::REMOTE_FIRST;
  if (has("TEMPI_ALLTOALLV_STAGED")) e.alltoallv = AlltoallvMethod::STAGED;
  if (has("TEMPI_ALLTOALLV_ISIR_STAGED")) e.alltoallv = AlltoallvMethod::ISIR_STAGED;
  if (has("TEMPI_ALLTOALLV_ISIR_REMOTE_STAGED")) e.alltoallv = AlltoallvMethod::ISIR_REMOTE_STAGED;
  if (has("TEMPI_NO_ALLTOALLV")) e.alltoallv = AlltoallvMethod::NONE;

  if (has("TEMPI_DATATYPE_ONESHOT")) e.datatype = DatatypeMethod::ONESHOT;
  if (has("TEMPI_DATATYPE_DEVICE")) e.datatype = DatatypeMethod::DEVICE;
  if (has("TEMPI_DATATYPE_STAGED")) e.datatype = DatatypeMethod::STAGED;
  if (has("TEMPI_DATATYPE_IPC")) e.datatype = DatatypeMethod::IPC;
  if (has("TEMPI_DATATYPE_AUTO")) e.datatype = DatatypeMethod::AUTO;

  // the reference's order (env.cpp:51-69): the last one present wins
  if (has("TEMPI_PLACEMENT_METIS") || has("TEMPI_PLACEMENT_KAHIP")) e.placement = PlacementMethod::PARTITION;
  if (has("TEMPI_PLACEMENT_RANDOM")) e.placement = PlacementMethod::RANDOM;

  if (has("TEMPI_CONTIGUOUS_STAGED")) e.contiguous = ContiguousMethod::STAGED;
  if (has("TEMPI_CONTIGUOUS_AUTO")) e.contiguous = ContiguousMethod::AUTO;

  if (const char *cd = std::getenv("TEMPI_CACHE_DIR")) {
    e.cacheDir = cd;
  } else if (const char *x = std::getenv("XDG_CACHE_HOME")) {
    e.cacheDir = std::string(x) + "/tempi";
  } else if (const char *h = std::getenv("HOME")) {
    e.cacheDir = std::string(h) + "/.tempi";
  } else {
    e.cacheDir = "/var/tmp";
  }

  if (const char *l = std::getenv("TEMPI_LOG_LEVEL")) {
    static const char *names[] = {"SPEW", "DEBUG", "INFO", "WARN", "ERROR", "FATAL"};
    for (int i = 0; i < 6; ++i)
      if (!strcasecmp(l, names[i])) logLevel = Level(i);
  }
  env = e;
}

void log_line(Level l, const std::string &msg) {
  static const char *names[] = {"SPEW", "DEBUG", "INFO", "WARN", "ERROR", "FATAL"};
  std::fprintf(stderr, "[tempi %s r%d] %s\n", names[int(l)], logRank, msg.c_str());
}

void fatal(const std::string &msg) {
  log_line(Level::FATAL, msg);
  std::fflush(stderr);
  std::abort();
}

} // namespace tempi
