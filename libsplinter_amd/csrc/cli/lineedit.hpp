// lineedit — line editing for the splinterctl REPL (the reference links linenoise:
// /root/reference/splinter_cli_main.c:832-872 and its completion callback at :446-510).
//
// On a terminal: raw-mode single-line editor with cursor movement (arrows, Home/End, Ctrl-A/E/B/F,
// Alt-B/F word moves), editing (Backspace, Delete, Ctrl-D, Ctrl-K/U/W/T), history (Up/Down,
// Ctrl-P/N), Tab completion cycling through the candidates of a callback, Ctrl-L clear screen and
// horizontal scrolling of lines wider than the terminal.  Not a terminal (pipes, tests) or
// TERM=dumb: a plain buffered read, so scripted use is unchanged.
#pragma once
#include <functional>
#include <string>
#include <vector>

namespace spl_le {

using Completer = std::function<void(const std::string& line, std::vector<std::string>& out)>;

enum class Read { Line, Eof, Interrupted };

// Read one line (without the newline) into `out`.  `history` is oldest-first; it is not modified.
Read read_line(const char* prompt, std::string& out, const std::vector<std::string>& history,
               const Completer& complete);

// true when read_line edits in raw mode (stdin and stdout are terminals and TERM is usable)
bool interactive();

}  // namespace spl_le
