// debug.cc — NCCL_DEBUG / NCCL_DEBUG_FILE logging, last-error buffer and NCCL_* parameter lookup.
//
// Reference behaviour: src/debug.cc:45-132 (levels VERSION/WARN/INFO/ABORT/TRACE, NCCL_DEBUG_FILE with
// %h/%p substitution), src/init.cc:3415-3443 (ncclGetLastError returns the last WARN text),
// src/misc/param.cc:54-111 (env first, then NCCL_CONF_FILE, ~/.nccl.conf, /etc/nccl.conf).
#include <dlfcn.h>
#include <errno.h>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <map>
#include <mutex>
#include <string>

#include "core.h"

namespace ncclamd {

int gLogLevel = -1;
static FILE* gLogFile = stderr;
static std::mutex gLogMutex;
static char gLastError[1024] = "";
static std::once_flag gLogOnce;

static void logInitOnce() {
  const char* lvl = getenv("NCCL_DEBUG");
  int level = LOG_NONE;
  if (lvl) {
    if (!strcasecmp(lvl, "VERSION")) level = LOG_VERSION;
    else if (!strcasecmp(lvl, "WARN")) level = LOG_WARN;
    else if (!strcasecmp(lvl, "INFO")) level = LOG_INFO;
    else if (!strcasecmp(lvl, "ABORT")) level = LOG_ABORT;
    else if (!strcasecmp(lvl, "TRACE")) level = LOG_TRACE;
  }
  const char* file = getenv("NCCL_DEBUG_FILE");
  if (file && level > LOG_NONE) {
    char path[4096];
    int o = 0;
    char host[256] = "";
    gethostname(host, sizeof(host) - 1);
    for (const char* p = file; *p && o < (int)sizeof(path) - 64; p++) {
      if (p[0] == '%' && p[1] == 'h') { o += snprintf(path + o, sizeof(path) - o, "%s", host); p++; }
      else if (p[0] == '%' && p[1] == 'p') { o += snprintf(path + o, sizeof(path) - o, "%d", getpid()); p++; }
      else path[o++] = *p;
    }
    path[o] = 0;
    FILE* f = fopen(path, "w");
    if (f) { setvbuf(f, nullptr, _IOLBF, 0); gLogFile = f; }
  }
  gLogLevel = level;
}

void logInit() { std::call_once(gLogOnce, logInitOnce); }

static const char* levelName(int l) {
  switch (l) {
    case LOG_WARN: return "WARN";
    case LOG_INFO: return "INFO";
    case LOG_TRACE: return "TRACE";
    default: return "";
  }
}

void logMessage(int level, const char* file, int line, const char* fmt, ...) {
  logInit();
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (level == LOG_WARN) {
    std::lock_guard<std::mutex> g(gLogMutex);
    snprintf(gLastError, sizeof(gLastError), "%s", buf);
  }
  if (gLogLevel < level) return;
  char host[64] = "";
  gethostname(host, sizeof(host) - 1);
  std::lock_guard<std::mutex> g(gLogMutex);
  if (level == LOG_WARN)
    fprintf(gLogFile, "%s:%d:%ld [%s] %s:%d NCCL %s %s\n", host, getpid(), (long)syscall(SYS_gettid),
            "mi355x", file, line, levelName(level), buf);
  else if (level == LOG_TRACE) {  // with a system-wide clock, so ranks' lines can be merged; flushed (a crash keeps them)
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    fprintf(gLogFile, "%s:%d:%ld %ld.%06ld NCCL %s %s\n", host, getpid(), (long)syscall(SYS_gettid), (long)ts.tv_sec,
            ts.tv_nsec / 1000, levelName(level), buf);
    fflush(gLogFile);
  } else {
    fprintf(gLogFile, "%s:%d:%ld NCCL %s %s\n", host, getpid(), (long)syscall(SYS_gettid), levelName(level), buf);
  }
}

void setLastError(const char* fmt, ...) {
  std::lock_guard<std::mutex> g(gLogMutex);
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(gLastError, sizeof(gLastError), fmt, ap);
  va_end(ap);
}

const char* lastError() { return gLastError; }

// ---------------------------------------------------------------- parameters
static std::map<std::string, std::string>* gConf = nullptr;
static std::once_flag gConfOnce;

static void loadConfFile(const char* path) {
  FILE* f = fopen(path, "r");
  if (!f) return;
  char line[1024];
  while (fgets(line, sizeof(line), f)) {
    char* s = line;
    while (*s == ' ' || *s == '\t') s++;
    if (*s == '#' || *s == '\n' || !*s) continue;
    char* eq = strchr(s, '=');
    if (!eq) continue;
    *eq = 0;
    char* v = eq + 1;
    char* end = v + strlen(v);
    while (end > v && (end[-1] == '\n' || end[-1] == ' ' || end[-1] == '\r')) *--end = 0;
    char* kend = eq;
    while (kend > s && (kend[-1] == ' ' || kend[-1] == '\t')) *--kend = 0;
    if (!gConf->count(s)) (*gConf)[s] = v;  // first file wins, env overrides all
  }
  fclose(f);
}

static void confInit() {
  gConf = new std::map<std::string, std::string>();
  const char* userFile = getenv("NCCL_CONF_FILE");
  if (userFile) loadConfFile(userFile);
  const char* home = getenv("HOME");
  if (home) {
    std::string p = std::string(home) + "/.nccl.conf";
    loadConfFile(p.c_str());
  }
  loadConfFile("/etc/nccl.conf");
}

const char* paramStr(const char* name) {
  const char* v = getenv(name);
  if (v) return v;
  std::call_once(gConfOnce, confInit);
  auto it = gConf->find(name);
  return it == gConf->end() ? nullptr : it->second.c_str();
}

int64_t paramInt(const char* name, int64_t deflt) {
  const char* v = paramStr(name);
  if (!v || !*v) return deflt;
  errno = 0;
  char* end = nullptr;
  long long x = strtoll(v, &end, 0);
  if (errno || end == v) {
    WARN("Invalid value %s for %s, using default %lld", v, name, (long long)deflt);
    return deflt;
  }
  return x;
}

// ---- roctx ranges (reference: NVTX ranges on the API entry points, src/collectives.cc:134,170,
// src/include/nvtx.h:125-137; payload = comm hash + message bytes). NCCL_AMD_ROCTX=1 resolves roctxRangePushA /
// roctxRangePop from rocprofiler-sdk's roctx library (the one rocprofv3 --marker-trace records; roctracer's
// libroctx64 as a fallback) at the first range; off, a range costs one load and branch.
int gRoctx = getenv("NCCL_AMD_ROCTX") && atoi(getenv("NCCL_AMD_ROCTX")) ? -1 : 0;  // -1: asked for, unresolved
static int (*gRangePush)(const char*) = nullptr;
static int (*gRangePop)() = nullptr;

static void roctxResolve() {
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      gRangePush = (int (*)(const char*))dlsym(h, "roctxRangePushA");
      gRangePop = (int (*)())dlsym(h, "roctxRangePop");
      if (gRangePush && gRangePop) {
        INFO("NCCL_AMD_ROCTX: roctx ranges through %s", lib);
        break;
      }
    }
    if (!gRangePush || !gRangePop) WARN("NCCL_AMD_ROCTX=1 but no roctx library could be loaded; no ranges");
    __atomic_store_n(&gRoctx, gRangePush && gRangePop ? 1 : 0, __ATOMIC_RELEASE);
  });
}

void RoctxRange::push(const char* fmt, ...) {
  if (gRoctx < 0) roctxResolve();
  on = gRoctx > 0;
  if (!on) return;
  char msg[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(msg, sizeof(msg), fmt, ap);
  va_end(ap);
  gRangePush(msg);
}

RoctxRange::~RoctxRange() {
  if (on) gRangePop();
}

}  // namespace ncclamd
