// lineedit.cpp — see lineedit.hpp.
#include "lineedit.hpp"

#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <strings.h>
#include <sys/ioctl.h>
#include <termios.h>
#include <unistd.h>

namespace spl_le {
namespace {

termios g_saved;
bool g_raw = false;
bool g_atexit = false;

void restore() {
  if (g_raw) {
    tcsetattr(STDIN_FILENO, TCSAFLUSH, &g_saved);
    g_raw = false;
  }
}

bool enable_raw() {
  if (tcgetattr(STDIN_FILENO, &g_saved) != 0) return false;
  if (!g_atexit) {
    atexit(restore);
    g_atexit = true;
  }
  termios t = g_saved;
  t.c_iflag &= ~(BRKINT | ICRNL | INPCK | ISTRIP | IXON);
  t.c_oflag &= ~OPOST;
  t.c_cflag |= CS8;
  t.c_lflag &= ~(ECHO | ICANON | IEXTEN | ISIG);
  t.c_cc[VMIN] = 1;
  t.c_cc[VTIME] = 0;
  if (tcsetattr(STDIN_FILENO, TCSAFLUSH, &t) != 0) return false;
  g_raw = true;
  return true;
}

int columns() {
  winsize ws;
  if (ioctl(STDOUT_FILENO, TIOCGWINSZ, &ws) == 0 && ws.ws_col > 0) return ws.ws_col;
  return 80;
}

void put(const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    const ssize_t n = write(STDOUT_FILENO, s.data() + off, s.size() - off);
    if (n <= 0) {
      if (n < 0 && errno == EINTR) continue;
      return;
    }
    off += (size_t)n;
  }
}

int read_byte() {
  unsigned char c;
  for (;;) {
    const ssize_t n = read(STDIN_FILENO, &c, 1);
    if (n == 1) return c;
    if (n < 0 && errno == EINTR) continue;
    return -1;
  }
}

struct Editor {
  std::string prompt, buf;
  size_t pos = 0;

  // one-line refresh: the window of `buf` around the cursor that fits after the prompt
  void refresh() {
    const size_t cols = (size_t)columns();
    const size_t plen = prompt.size();
    size_t start = 0, len = buf.size(), cur = pos;
    while (plen + cur >= cols && start < buf.size()) {
      ++start;
      --cur;
      --len;
    }
    while (plen + len > cols && len > 0) --len;
    std::string s = "\r" + prompt + buf.substr(start, len) + "\x1b[0K\r";
    if (plen + cur) s += "\x1b[" + std::to_string(plen + cur) + "C";
    put(s);
  }
  void insert(char c) {
    buf.insert(pos++, 1, c);
    refresh();
  }
  void word_left() {
    while (pos > 0 && buf[pos - 1] == ' ') --pos;
    while (pos > 0 && buf[pos - 1] != ' ') --pos;
  }
  void word_right() {
    while (pos < buf.size() && buf[pos] == ' ') ++pos;
    while (pos < buf.size() && buf[pos] != ' ') ++pos;
  }
};

}  // namespace

bool interactive() {
  if (!isatty(STDIN_FILENO) || !isatty(STDOUT_FILENO)) return false;
  const char* term = getenv("TERM");
  return !(term && (!strcasecmp(term, "dumb") || !strcasecmp(term, "cons25") || !strcasecmp(term, "emacs")));
}

Read read_line(const char* prompt, std::string& out, const std::vector<std::string>& history,
               const Completer& complete) {
  out.clear();
  if (!interactive() || !enable_raw()) {
    fputs(prompt, stderr);
    fflush(stderr);
    char b[65536];
    if (!fgets(b, sizeof b, stdin)) return Read::Eof;
    out = b;
    while (!out.empty() && (out.back() == '\n' || out.back() == '\r')) out.pop_back();
    return Read::Line;
  }
  Editor e;
  e.prompt = prompt;
  // history browsing works on a copy with the line being edited as its newest entry
  std::vector<std::string> hist(history);
  hist.push_back("");
  size_t hidx = hist.size() - 1;
  e.refresh();
  Read result = Read::Line;
  for (;;) {
    int c = read_byte();
    if (c < 0) {
      result = Read::Eof;
      break;
    }
    if (c == '\t' && complete) {
      std::vector<std::string> cands;
      complete(e.buf, cands);
      if (cands.empty()) {
        put("\x07");
        continue;
      }
      // cycle: Tab shows the next candidate, Esc restores the line, any other key keeps the shown one
      const std::string orig = e.buf;
      const size_t opos = e.pos;
      size_t i = 0;
      for (;;) {
        e.buf = i < cands.size() ? cands[i] : orig;
        e.pos = i < cands.size() ? e.buf.size() : opos;
        e.refresh();
        c = read_byte();
        if (c == '\t') {
          i = (i + 1) % (cands.size() + 1);
          if (i == cands.size()) put("\x07");
          continue;
        }
        if (c == 27) {
          e.buf = orig;
          e.pos = opos;
          e.refresh();
          c = 0;  // consumed
        }
        break;
      }
      if (c <= 0) continue;
      // fall through: the key that ended the cycle is processed normally
    }
    switch (c) {
      case 13:
      case 10:
        hist.pop_back();
        out = e.buf;
        put("\r\n");
        restore();
        return Read::Line;
      case 3:  // Ctrl-C
        put("^C\r\n");
        restore();
        return Read::Interrupted;
      case 4:  // Ctrl-D: EOF on an empty line, else delete under the cursor
        if (e.buf.empty()) {
          put("\r\n");
          restore();
          return Read::Eof;
        }
        if (e.pos < e.buf.size()) {
          e.buf.erase(e.pos, 1);
          e.refresh();
        }
        break;
      case 127:
      case 8:  // Backspace
        if (e.pos > 0) {
          e.buf.erase(--e.pos, 1);
          e.refresh();
        }
        break;
      case 1: e.pos = 0; e.refresh(); break;              // Ctrl-A
      case 5: e.pos = e.buf.size(); e.refresh(); break;   // Ctrl-E
      case 2: if (e.pos > 0) --e.pos; e.refresh(); break;   // Ctrl-B
      case 6: if (e.pos < e.buf.size()) ++e.pos; e.refresh(); break;  // Ctrl-F
      case 11: e.buf.erase(e.pos); e.refresh(); break;     // Ctrl-K
      case 21: e.buf.clear(); e.pos = 0; e.refresh(); break;  // Ctrl-U
      case 23: {  // Ctrl-W: delete the previous word
        const size_t end = e.pos;
        e.word_left();
        e.buf.erase(e.pos, end - e.pos);
        e.refresh();
        break;
      }
      case 20:  // Ctrl-T: transpose
        if (e.pos > 0 && e.buf.size() > 1) {
          if (e.pos == e.buf.size()) --e.pos;
          std::swap(e.buf[e.pos - 1], e.buf[e.pos]);
          ++e.pos;
          e.refresh();
        }
        break;
      case 12: put("\x1b[H\x1b[2J"); e.refresh(); break;  // Ctrl-L
      case 16:  // Ctrl-P
      case 14:  // Ctrl-N
      history_move: {
        const bool up = c == 16;
        if (hist.size() > 1) {
          hist[hidx] = e.buf;
          if (up && hidx > 0) --hidx;
          else if (!up && hidx + 1 < hist.size()) ++hidx;
          e.buf = hist[hidx];
          e.pos = e.buf.size();
          e.refresh();
        }
        break;
      }
      case 27: {  // escape sequences
        const int s0 = read_byte();
        if (s0 < 0) break;
        if (s0 == 'b' || s0 == 'f') {  // Alt-B / Alt-F
          if (s0 == 'b') e.word_left();
          else e.word_right();
          e.refresh();
          break;
        }
        const int s1 = read_byte();
        if (s1 < 0) break;
        if (s0 == '[' && s1 >= '0' && s1 <= '9') {
          const int s2 = read_byte();
          if (s2 == '~') {
            if (s1 == '3' && e.pos < e.buf.size()) {  // Delete
              e.buf.erase(e.pos, 1);
              e.refresh();
            } else if (s1 == '1' || s1 == '7') {
              e.pos = 0;
              e.refresh();
            } else if (s1 == '4' || s1 == '8') {
              e.pos = e.buf.size();
              e.refresh();
            }
          }
          break;
        }
        if (s0 == '[' || s0 == 'O') {
          switch (s1) {
            case 'A': c = 16; goto history_move;
            case 'B': c = 14; goto history_move;
            case 'C': if (e.pos < e.buf.size()) ++e.pos; e.refresh(); break;
            case 'D': if (e.pos > 0) --e.pos; e.refresh(); break;
            case 'H': e.pos = 0; e.refresh(); break;
            case 'F': e.pos = e.buf.size(); e.refresh(); break;
          }
        }
        break;
      }
      default:
        if (c >= 32) e.insert((char)c);
        break;
    }
  }
  restore();
  return result;
}

}  // namespace spl_le
