// Declaration-only stand-in for {fmt}'s core API as utils/flog.h uses it (fmt 9+: format_string,
// string_view, format), used ONLY by tests/test_overlay_syntax.py's `g++ -fsyntax-only` of the
// overlay inside the reference tree ({fmt} is not installed in this image). Nothing is defined,
// linked or run.
#pragma once
#include <string>
#include <string_view>
#include <type_traits>
namespace fmt {
using string_view = std::string_view;
template <class... Args>
struct basic_format_string {
    template <class S, class = std::enable_if_t<std::is_convertible_v<const S&, std::string_view>>>
    basic_format_string(const S& s);
    operator string_view() const;
};
template <class T> struct type_identity { using type = T; };
template <class... Args>
using format_string = basic_format_string<typename type_identity<Args>::type...>;
template <class... Args>
std::string format(format_string<Args...> fmt, Args&&... args);
}  // namespace fmt
