// sidecar — terminal monitor: host CPU / memory history, GPU telemetry, and the
// debug chatter of a store (keys labelled with the debug bloom bit) or a tailed
// text file.  Same usage, keys and label contract as the reference tool
// (/root/reference/sidecar.c:1-25 usage, :89-131 debug ring + label watch,
// :390-590 main loop, keystroke jobs :456-484):
//
//   sidecar [spl:STORE | FILE] [--once] [--interval-ms N]
//
//   * spl:STORE  attaches to a store (shm name, file path or hbm:NAME), binds
//     the debug label 0x0800000000000000 to signal group 63 and shows the value
//     of every labelled key whenever that group pulses;
//   * FILE       tails a text file;
//   * keys 0-9   run ./.sidecar.N (must be a symlink) as a background job and
//     report its exit code; q quits.
//   * GPU panel  (new): per-card busy %, VRAM use, temperature and power from
//     the amdgpu sysfs/hwmon files, so the monitor shows the MI355X side of a
//     splinference / bench run.
//   * --once     renders a single frame without raw mode (scripts, tests).
// Jobs are started with posix_spawn (no fork+exec of this process image).
#include <cerrno>
#include <cmath>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <dirent.h>
#include <fcntl.h>
#include <spawn.h>
#include <string>
#include <sys/ioctl.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <termios.h>
#include <unistd.h>
#include <vector>

#include "splinter_ext.h"

extern char** environ;

namespace {

constexpr uint64_t kDebugBloom = 0x0800000000000000ull;
constexpr unsigned kDebugGroup = 63;
constexpr int kHistH = 10, kMaxW = 512, kMaxDebug = 64;

struct Cpu {
  unsigned long long v[8] = {};
};

int g_cols = 80, g_rows = 24, g_graph = 50;
volatile sig_atomic_t g_resize = 0;
termios g_orig;
bool g_raw = false;
std::deque<std::string> g_debug;
double g_io = 0.0;

void debug_append(const std::string& s) {
  g_debug.push_back(s);
  while ((int)g_debug.size() > kMaxDebug) g_debug.pop_front();
}

void restore_term() {
  if (g_raw) tcsetattr(STDIN_FILENO, TCSAFLUSH, &g_orig);
}

void raw_mode() {
  if (tcgetattr(STDIN_FILENO, &g_orig) != 0) return;
  termios r = g_orig;
  r.c_lflag &= ~(ECHO | ICANON);
  r.c_cc[VMIN] = 0;
  r.c_cc[VTIME] = 0;
  tcsetattr(STDIN_FILENO, TCSAFLUSH, &r);
  g_raw = true;
  atexit(restore_term);
}

void on_winch(int) {
  winsize ws;
  if (ioctl(STDOUT_FILENO, TIOCGWINSZ, &ws) == 0 && ws.ws_col > 0) {
    g_cols = ws.ws_col;
    g_rows = ws.ws_row;
  }
  g_graph = std::max(20, std::min(kMaxW, g_cols - 12));
  g_resize = 1;
}

Cpu read_cpu() {
  Cpu c;
  if (FILE* f = fopen("/proc/stat", "r")) {
    if (fscanf(f, "cpu %llu %llu %llu %llu %llu %llu %llu %llu", &c.v[0], &c.v[1], &c.v[2], &c.v[3], &c.v[4], &c.v[5],
               &c.v[6], &c.v[7]) != 8)
      c = Cpu{};
    fclose(f);
  }
  return c;
}

double cpu_pct(Cpu& prev) {
  const Cpu cur = read_cpu();
  auto idle = [](const Cpu& c) { return c.v[3] + c.v[4]; };
  auto busy = [](const Cpu& c) { return c.v[0] + c.v[1] + c.v[2] + c.v[5] + c.v[6] + c.v[7]; };
  const unsigned long long dt = (idle(cur) + busy(cur)) - (idle(prev) + busy(prev));
  const unsigned long long di = idle(cur) - idle(prev), dio = cur.v[4] - prev.v[4];
  prev = cur;
  if (!dt) { g_io = 0; return 0; }
  g_io = 100.0 * (double)dio / (double)dt;
  return 100.0 * (double)(dt - di) / (double)dt;
}

double mem_pct(double* swap) {
  unsigned long tot = 1, fr = 0, buf = 0, cac = 0, st = 0, sf = 0;
  if (FILE* f = fopen("/proc/meminfo", "r")) {
    char k[64];
    unsigned long v;
    char u[16];
    while (fscanf(f, "%63s %lu %15s\n", k, &v, u) >= 2) {
      if (!strcmp(k, "MemTotal:")) tot = v;
      else if (!strcmp(k, "MemFree:")) fr = v;
      else if (!strcmp(k, "Buffers:")) buf = v;
      else if (!strcmp(k, "Cached:")) cac = v;
      else if (!strcmp(k, "SwapTotal:")) st = v;
      else if (!strcmp(k, "SwapFree:")) sf = v;
    }
    fclose(f);
  }
  *swap = st ? 100.0 * (double)(st - sf) / (double)st : 0.0;
  return 100.0 * (double)(tot - fr - buf - cac) / (double)tot;
}

long read_long(const std::string& p) {
  long v = -1;
  if (FILE* f = fopen(p.c_str(), "r")) {
    if (fscanf(f, "%ld", &v) != 1) v = -1;
    fclose(f);
  }
  return v;
}

struct Gpu {
  std::string card;
  long busy = -1, vram_used = -1, vram_total = -1, temp_mc = -1, power_uw = -1;
};

std::vector<Gpu> read_gpus() {
  std::vector<Gpu> out;
  DIR* d = opendir("/sys/class/drm");
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    if (strncmp(e->d_name, "card", 4) || strchr(e->d_name, '-')) continue;
    const std::string dev = std::string("/sys/class/drm/") + e->d_name + "/device";
    Gpu g;
    g.card = e->d_name;
    g.busy = read_long(dev + "/gpu_busy_percent");
    g.vram_used = read_long(dev + "/mem_info_vram_used");
    g.vram_total = read_long(dev + "/mem_info_vram_total");
    if (g.busy < 0 && g.vram_total < 0) continue;  // not an amdgpu device
    if (DIR* h = opendir((dev + "/hwmon").c_str())) {
      while (dirent* he = readdir(h)) {
        if (strncmp(he->d_name, "hwmon", 5)) continue;
        const std::string hp = dev + "/hwmon/" + he->d_name;
        g.temp_mc = read_long(hp + "/temp1_input");
        g.power_uw = read_long(hp + "/power1_average");
        if (g.power_uw < 0) g.power_uw = read_long(hp + "/power1_input");
      }
      closedir(h);
    }
    out.push_back(g);
  }
  closedir(d);
  return out;
}

void bar(const char* label, double pct) {
  const int filled = (int)(pct / 100.0 * g_graph);
  fputs("┌> ", stdout);
  for (int i = 0; i < g_graph; ++i) fputs(i < filled ? "■" : " ", stdout);
  printf("%-3s\n└> %-5.1f%%\n", label, pct);
}

}  // namespace

int main(int argc, char** argv) {
  std::string target, store;
  bool once = false;
  int interval_ms = 500;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--once")) once = true;
    else if (!strcmp(argv[i], "--interval-ms") && i + 1 < argc) interval_ms = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-h") || !strcmp(argv[i], "--help")) {
      printf("Usage: %s [spl:STORE | FILE] [--once] [--interval-ms N]\n", argv[0]);
      return 0;
    } else target = argv[i];
  }
  FILE* tail = nullptr;
  if (!target.empty()) {
    if (!strncmp(target.c_str(), "spl:", 4)) {
      store = target.substr(4);
      if (splinter_open_or_create(store.c_str(), 1024, 4096) != 0) {
        fprintf(stderr, "Unable to open splinter store: %s\n", store.c_str());
        perror("splinter_open_or_create()");
        return 1;
      }
      if (splinter_watch_label_register(kDebugBloom, kDebugGroup) != 0) fprintf(stderr, "* spl:watch(!)\n");
    } else if (!(tail = fopen(target.c_str(), "r"))) {
      fprintf(stderr, "Unable to load debug file %s\n", target.c_str());
      perror("file");
    } else {
      setvbuf(tail, nullptr, _IONBF, 0);
      if (!once) fseek(tail, 0, SEEK_END);
    }
  }
  if (!once) {
    raw_mode();
    struct sigaction sa {};
    sa.sa_handler = on_winch;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_RESTART;
    sigaction(SIGWINCH, &sa, nullptr);
  }
  on_winch(0);

  std::vector<double> hcpu(kMaxW, 0.0), hmem(kMaxW, 0.0);
  Cpu prev = read_cpu();
  uint64_t last_sig = store.empty() ? 0 : splinter_get_signal_count(kDebugGroup);
  if (!store.empty() && once) last_sig = ~0ull;  // one-shot: show the current labelled keys
  pid_t jobs[10] = {};
  std::string results[10];
  int tick = 0;
  if (!once) printf("\033[2J");
  for (;;) {
    for (int i = 0; i < 10; ++i) {
      int st;
      if (jobs[i] > 0 && waitpid(jobs[i], &st, WNOHANG) > 0) {
        results[i] = ".sidecar." + std::to_string(i) + ":" + std::to_string(WIFEXITED(st) ? WEXITSTATUS(st) : -1);
        jobs[i] = 0;
      }
    }
    char c;
    while (!once && read(STDIN_FILENO, &c, 1) == 1) {
      if (c >= '0' && c <= '9') {
        const int idx = c - '0';
        const std::string script = ".sidecar." + std::to_string(idx);
        struct stat sb;
        if (jobs[idx] == 0 && lstat(script.c_str(), &sb) == 0 && S_ISLNK(sb.st_mode)) {
          posix_spawn_file_actions_t fa;
          posix_spawn_file_actions_init(&fa);
          posix_spawn_file_actions_addopen(&fa, STDOUT_FILENO, "/dev/null", O_WRONLY, 0);
          posix_spawn_file_actions_addopen(&fa, STDERR_FILENO, "/dev/null", O_WRONLY, 0);
          const std::string path = "./" + script;
          char* const args[] = {(char*)"sh", (char*)"-c", (char*)path.c_str(), nullptr};
          pid_t pid;
          if (posix_spawn(&pid, "/bin/sh", &fa, nullptr, args, environ) == 0) {
            jobs[idx] = pid;
            results[idx].clear();
          }
          posix_spawn_file_actions_destroy(&fa);
        }
      } else if (c == 'q' || c == 'Q') {
        printf("\033[2J\033[H");
        splinter_close();
        return 0;
      }
    }
    double swap = 0;
    const double cpu = cpu_pct(prev), mem = mem_pct(&swap);
    double l1 = 0, l5 = 0, l15 = 0;
    int run = 0, total = 0;
    if (FILE* f = fopen("/proc/loadavg", "r")) {
      if (fscanf(f, "%lf %lf %lf %d/%d", &l1, &l5, &l15, &run, &total) != 5) l1 = l5 = l15 = 0;
      fclose(f);
    }
    bool redraw = false;
    if (tail) {
      char line[1024];
      while (fgets(line, sizeof line, tail)) {
        line[strcspn(line, "\r\n")] = 0;
        debug_append(line);
        redraw = true;
      }
      clearerr(tail);
    }
    if (!store.empty()) {
      const uint64_t sig = splinter_get_signal_count(kDebugGroup);
      if (sig != last_sig) {
        splinter_enumerate_matches(
            kDebugBloom,
            [](const char* key, uint64_t epoch, void*) {
              if (!key) return;
              std::vector<char> buf(65536, 0);
              size_t n = 0;
              const int rc = splinter_get(key, buf.data(), buf.size() - 1, &n);
              char msg[kMaxW];
              snprintf(msg, sizeof msg, "(%lu) %s", (unsigned long)epoch, rc == 0 ? buf.data() : "(no value set)");
              debug_append(msg);
            },
            nullptr);
        redraw = true;
      }
      last_sig = sig;
    }
    if (tick == 0) {
      hcpu.erase(hcpu.begin());
      hcpu.push_back(cpu);
      hmem.erase(hmem.begin());
      hmem.push_back(mem);
    }
    tick = (tick + 1) % 4;
    if (!once) {
      if (g_resize || redraw) { printf("\033[2J"); g_resize = 0; }
      printf("\033[H");
    }
    printf("History (CPU=█, RAM=░)\n");
    for (int row = kHistH; row >= 0; --row) {
      for (int col = kMaxW - g_graph; col < kMaxW; ++col) {
        const int cc = (int)(hcpu[col] / 100.0 * kHistH), mm = (int)(hmem[col] / 100.0 * kHistH);
        fputs(cc >= row && mm >= row ? "▓" : cc >= row ? "█" : mm >= row ? "░" : " ", stdout);
      }
      putchar('\n');
    }
    putchar('\n');
    bar("cpu", cpu);
    printf(" > s=%-.1f%% | i=%-.1f%% | 1=%-.2f | 5=%-.2f | 15=%-.2f\n", swap, g_io, l1, l5, l15);
    printf(" > [%d/%d]\n", run, total);
    bar("mem", mem);
    for (const Gpu& g : read_gpus()) {
      printf(" > %s busy=%ld%% vram=%.1f/%.1f GiB temp=%.0fC power=%.0fW\n", g.card.c_str(), g.busy,
             g.vram_used / 1073741824.0, g.vram_total / 1073741824.0, g.temp_mc / 1000.0, g.power_uw / 1e6);
    }
    if (!store.empty()) {
      spl_store* s = spl_store_current();
      uint32_t slots = 0, mv = 0, stride = 0;
      spl_store_geometry(s, &slots, &mv, &stride);
      printf(" > bus: %s (%s, %u slots) group %u pulses=%lu\n", store.c_str(), spl_store_backend(s), slots,
             kDebugGroup, (unsigned long)last_sig);
    } else if (tail) {
      printf(" > tail: %s\n", target.c_str());
    }
    const int avail = std::max(0, g_rows - (kHistH + 12));
    const int start = (int)g_debug.size() > avail ? (int)g_debug.size() - avail : 0;
    for (int i = once ? 0 : start; i < (int)g_debug.size(); ++i)
      printf("%.*s\n", g_cols > 1 ? g_cols - 1 : 1, g_debug[(size_t)i].c_str());
    for (int i = 0; i < 10; ++i)
      if (!results[i].empty()) printf("Job result: %s\n", results[i].c_str());
    if (!once) printf("\033[J");
    fflush(stdout);
    if (once) break;
    usleep((useconds_t)interval_ms * 1000);
  }
  splinter_close();
  return 0;
}
