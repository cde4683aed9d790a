// diag.cpp — per-thread record of the latest failed library call.
//
// mccsCommSetupRank / mccsCommConnect / mccsCommInitAll fold a few dozen
// runtime calls into one result code (as the reference's init path does:
// proxy/engine.rs:220-621, comm/device.rs:81-183).  A failing call records
// here which step it was in and which runtime call failed with which
// hipError_t, so a caller (ipc_worker.py, the bench, a Rust service) can
// print the cause instead of "unhandled HIP error".
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "comm.h"

namespace mccs {
namespace {
thread_local std::vector<std::string> t_steps;
thread_local std::string t_last;
thread_local int t_last_hip = 0;

std::string step_path() {
  std::string s;
  for (const auto& n : t_steps) {
    if (!s.empty()) s += " > ";
    s += n;
  }
  return s;
}

const char* base_name(const char* file) {
  const char* b = std::strrchr(file, '/');
  return b ? b + 1 : file;
}

// "rt().HostMallocMapped((void**)&c->h_work, ...)" -> "HostMallocMapped";
// "hipIpcGetMemHandle(&h.ipc, p)" -> "hipIpcGetMemHandle"
std::string call_name(const char* call) {
  std::string s(call);
  if (s.rfind("rt().", 0) == 0) s = s.substr(5);
  const size_t p = s.find('(');
  return p == std::string::npos ? s : s.substr(0, p);
}
}  // namespace

StepScope::StepScope(std::string name) { t_steps.push_back(std::move(name)); }
StepScope::~StepScope() { t_steps.pop_back(); }

void err_clear() {
  t_last.clear();
  t_last_hip = 0;
}

void err_hip(const char* call, hipError_t e, const char* file, int line) {
  // the failure travels in the result and this record; no sticky copy stays
  // on the thread for the caller's next hipGetLastError() to find
  (void)hipGetLastError();
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s: %s -> %s (%s) at %s:%d", step_path().c_str(), call_name(call).c_str(),
                hipGetErrorName(e), hipGetErrorString(e), base_name(file), line);
  t_last = buf;
  t_last_hip = (int)e;
  MCCS_LOG("%s", buf);
}

void err_note(const char* file, int line, const char* fmt, ...) {
  char msg[384];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(msg, sizeof(msg), fmt, ap);
  va_end(ap);
  char buf[640];
  std::snprintf(buf, sizeof(buf), "%s: %s at %s:%d", step_path().c_str(), msg, base_name(file), line);
  t_last = buf;
  t_last_hip = 0;
  MCCS_LOG("%s", buf);
}

}  // namespace mccs

extern "C" const char* mccsGetLastErrorString(void) { return mccs::t_last.c_str(); }
extern "C" int mccsGetLastHipError(void) { return mccs::t_last_hip; }
