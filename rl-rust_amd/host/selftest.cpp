// selftest — host-only checks of the CLI helpers (no GPU): prints
// moving_average / rust_f64 / rust_duration results for tests/test_cli.py.
#include "cli_common.hpp"

int main() {
    const std::vector<double> v = {1, 2, 3, 4, 5, 6, 7};
    for (size_t w : {1, 2, 3, 7, 10}) {
        std::printf("ma %zu:", w);
        for (double x : cli::moving_average(w, v)) std::printf(" %s", cli::rust_f64(x).c_str());
        std::printf("\n");
    }
    for (double x : {0.0, 1.0, 0.1, 1e-7, 123456789.125, -2.5, 1.0 / 3.0})
        std::printf("f64 %s\n", cli::rust_f64(x).c_str());
    for (long long ns : {999LL, 1500LL, 2500000LL, 3210000000LL})
        std::printf("dur %s\n", cli::rust_duration(std::chrono::nanoseconds(ns)).c_str());
    return 0;
}
