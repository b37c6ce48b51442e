// main.cpp — the mcaat CLI over the MI355X hot path. Mirrors the release main of the
// reference (src/main.cpp:496-591): settings check, SDBG build, CycleFinder, relevant reads
// (step 6), spacer ordering (step 7), results / benchmark (step 8) and CRISPRAnalyzer, which
// writes settings.output_file (CRISPR_Arrays.txt). The cycles themselves are also written to
// <cycles_folder>/cycles.txt (not in the reference's release build).
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <csignal>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <random>
#include <sstream>
#include <thread>

#include "downstream.h"

namespace fs = std::filesystem;

static bool check_for_error(Settings &settings) {  // main.cpp:50-59
    std::cout << "Step 1. Checking the inputs: " << std::endl;
    std::string bad = settings.print_settings();
    if (bad.empty()) {
        std::cout << "All inputs are correct. [✔]" << std::endl;
        return false;
    }
    std::cout << "Please check the following: " << bad << std::endl;
    return true;
}

static std::string cycle_sequence(const SDBG &sdbg, const std::vector<uint64_t> &cycle) {
    std::vector<uint8_t> lab(sdbg.k());
    std::string s;
    for (size_t i = 0; i < cycle.size(); ++i) {
        sdbg.GetLabel(cycle[i], lab.data());
        if (i == 0) for (int j = 0; j < sdbg.k(); ++j) s += "ACGT"[lab[j] - 1];
        else s += "ACGT"[lab[sdbg.k() - 1] - 1];
    }
    return s;
}

// Multi-GPU run (--gpus N): rank 0 forks ranks 1..N-1 before anything touches the GPU, one
// process per GPU. The RCCL id goes to each child through a pipe; the shared-memory transport
// needs only the segment name chosen here. Ranks other than 0 print nothing to stdout and end
// after step 6 (the relevant reads are gathered to every rank); rank 0 writes the outputs. A
// rank that fails ends the whole run (a watcher thread on rank 0 reaps the children).
struct Ranks {
    std::vector<pid_t> children;
    std::vector<int> to_child;  // rank 0: write ends of the id pipes
    int from_parent = -1;       // rank > 0: read end
    std::string shm_name;
    std::thread watcher;

    ~Ranks() {
        if (watcher.joinable()) watcher.detach();  // an error path: the process is ending
    }
    void kill_children() {
        for (pid_t p : children) kill(p, SIGTERM);
    }
    static void write_all(int fd, const void *p, size_t n) {
        const char *c = (const char *)p;
        while (n) {
            const ssize_t w = write(fd, c, n);
            if (w <= 0) throw std::runtime_error("multi-GPU: cannot pass the communicator id to a rank");
            c += w;
            n -= (size_t)w;
        }
    }
    static void read_all(int fd, void *p, size_t n) {
        char *c = (char *)p;
        while (n) {
            const ssize_t r = read(fd, c, n);
            if (r <= 0) throw std::runtime_error("multi-GPU: rank 0 ended before passing the communicator id");
            c += r;
            n -= (size_t)r;
        }
    }

    void fork_ranks(Settings &s) {
        std::random_device rd;
        char name[64];
        snprintf(name, sizeof name, "/mcaat_%d_%08x", (int)getpid(), (unsigned)rd());
        shm_name = name;
        std::cout.flush();
        fflush(stdout);
        for (int r = 1; r < s.gpus; ++r) {
            int fds[2];
            if (pipe(fds) != 0) throw std::runtime_error("multi-GPU: pipe failed");
            const pid_t pid = fork();
            if (pid < 0) throw std::runtime_error("multi-GPU: fork failed");
            if (pid == 0) {
                close(fds[1]);
                for (int w : to_child) close(w);
                to_child.clear();
                children.clear();
                from_parent = fds[0];
                s.rank = r;
                if (!freopen("/dev/null", "w", stdout)) throw std::runtime_error("multi-GPU: cannot silence a rank");
                return;
            }
            close(fds[0]);
            children.push_back(pid);
            to_child.push_back(fds[1]);
        }
    }

    // after fork: this rank's context and communicator
    void connect(Settings &s) {
        mcaat_ctx *ctx = mcaat_host_ctx(mcaat_rank_device(s));
        if (s.comm == "rccl") {
            int n = 0;
            mcaat_check(mcaat_device_count(&n), "mcaat_device_count");
            if (s.gpus > n)
                throw std::runtime_error("--gpus " + std::to_string(s.gpus) + " > " + std::to_string(n) +
                                         " visible GPUs (RCCL needs one GPU per rank; --comm shm shares GPUs)");
            uint8_t id[MCAAT_COMM_ID_BYTES];
            if (s.rank == 0) {
                mcaat_check(mcaat_comm_unique_id(id), "mcaat_comm_unique_id");
                for (int w : to_child) write_all(w, id, sizeof id);
            } else {
                read_all(from_parent, id, sizeof id);
            }
            mcaat_check(mcaat_comm_init_rccl(ctx, s.gpus, s.rank, id, &s.mcomm), "joining the ranks (RCCL)");
        } else {
            mcaat_check(mcaat_comm_init_shm(ctx, s.gpus, s.rank, shm_name.c_str(), 0, &s.mcomm),
                        "joining the ranks (shared memory)");
        }
        for (int w : to_child) close(w);
        to_child.clear();
        if (from_parent >= 0) close(from_parent);
        from_parent = -1;
    }

    void watch() {
        std::vector<pid_t> kids = children;
        watcher = std::thread([kids]() {
            // whichever rank ends first is reaped first (a failure of rank 3 is seen while rank
            // 1 is still running); only the rank pids are waited on, so another child of rank 0
            // (a popen, a system()) keeps its own exit status
            std::vector<bool> done(kids.size(), false);
            for (size_t left = kids.size(); left > 0;) {
                bool reaped = false;
                for (size_t r = 0; r < kids.size(); ++r) {
                    if (done[r]) continue;
                    int st = 0;
                    const pid_t p = waitpid(kids[r], &st, WNOHANG);
                    if (p == 0 || (p < 0 && errno == EINTR)) continue;
                    done[r] = true;
                    --left;
                    reaped = true;
                    if (p < 0) continue;  // not ours any more (ECHILD)
                    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) {
                        std::cerr << "rank " << r + 1 << " failed; ending the run" << std::endl;
                        for (pid_t q : kids) kill(q, SIGTERM);
                        _exit(1);
                    }
                }
                if (!reaped) std::this_thread::sleep_for(std::chrono::milliseconds(20));
            }
        });
    }
};

static void banner(const char *title) {
    std::cout << "\n══════════════════════════════════════════════" << std::endl;
    std::cout << title << std::endl;
    std::cout << "══════════════════════════════════════════════" << std::endl;
}

static int run(Settings &settings, Ranks &ranks);

using Clock = std::chrono::steady_clock;
static Clock::time_point g_main_start;
static double since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

int main(int argc, char **argv) {
    g_main_start = Clock::now();
    try {
        Settings settings = parse_arguments(argc, argv);
        if (check_for_error(settings)) {  // main.cpp:499-513
            std::cout << "Folder " << settings.output_folder << " will be deleted due to errors." << std::endl;
            std::cout << "Do you want that folder to be removed? (y/n): ";
            char answer = 'n';
            std::cin >> answer;
            if (answer != 'y' && answer != 'Y') {
                std::cout << "Exiting the program." << std::endl;
                return 1;
            }
            std::cout << "Removing folder: " << settings.output_folder << std::endl;
            fs::remove_all(settings.output_folder);
            return 1;
        }
        Ranks ranks;
        if (settings.gpus > 1) {
            ranks.fork_ranks(settings);  // before any GPU call
            // rank 0 reaps the children from here on: a rank that dies before it joins the
            // communicator (ncclCommInitRank has no timeout) ends the run instead of hanging it
            if (settings.rank == 0) ranks.watch();
        }
        try {
            return run(settings, ranks);
        } catch (...) {
            ranks.kill_children();
            throw;
        }
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return 1;
    }
}

static int run(Settings &settings, Ranks &ranks) {
    const bool rank0 = settings.rank == 0;
    {
        // brings the HIP runtime up before the timed span (errors surface in SDBGBuild, after
        // it has written data.lib as the reference does)
        int n_dev = 0;
        (void)mcaat_device_count(&n_dev);
        // and loads the kernels' code objects (HIP otherwise loads each file's at the first launch
        // of one of its kernels, inside the span); MCAAT_PRELOAD=0 leaves that to HIP
        const char *pl = getenv("MCAAT_PRELOAD");
        if (n_dev > 0 && !(pl && pl[0] == '0')) {
            (void)mcaat_preload(mcaat_rank_device(settings));
            // the rank's GPU context (its streams) is set up with the runtime as well
            if (settings.gpus <= 1) (void)mcaat_host_ctx(mcaat_rank_device(settings));
        }
    }
    if (settings.gpus > 1) {
        if (const char *e = getenv("MCAAT_TEST_RANK_EXIT"))  // test hook: this rank dies before joining
            if (atoi(e) == settings.rank && settings.rank > 0) _exit(3);
        ranks.connect(settings);
    }
    {
        using clk = std::chrono::steady_clock;
        const double t_span_start = since(g_main_start);
        const auto t_start = clk::now();
        SDBGBuild sdbg_build(settings);                        // main.cpp:517
        const auto t_built = clk::now();
        SDBG sdbg;                                             // main.cpp:522-530
        sdbg.LoadFromDevice(sdbg_build.release_graph());
        std::cout << "Loaded the graph" << std::endl;
        settings.sdbg = &sdbg;
        std::cout << "FBCE START:" << std::endl;
        CycleFinder cycle_finder(settings);                    // main.cpp:536
        {
            // the reference's hot-path span, SDBGBuild start -> CycleFinder end (main.cpp:517-536)
            const auto t_end = clk::now();
            auto sec = [](clk::duration d) { return std::chrono::duration<double>(d).count(); };
            char line[256];
            snprintf(line, sizeof line,
                     "TIMING span_s=%.6f sdbg_build_s=%.6f build_lib_s=%.6f cycle_finder_s=%.6f",
                     sec(t_end - t_start), sec(t_built - t_start), sdbg_build.lib_seconds, sec(t_end - t_built));
            std::cout << line << std::endl;
        }
        const double t_span_end = since(g_main_start);
        // a graph built and searched per shard is gathered on every rank for the steps after
        // the span (read mapping, spacer ordering read the whole graph); no-op on one GPU
        if (settings.gpus > 1 && settings.mcomm) {
            int sharded = 0;
            mcaat_check(mcaat_graph_shard_info(sdbg.device(), &sharded, nullptr, nullptr), "graph shard info");
            if (sharded) {
                mcaat_check(mcaat_graph_unshard(sdbg.device(), settings.mcomm), "gathering the sharded graph");
                sdbg.SyncFromDevice();
            }
        }
        auto cycles_map = cycle_finder.results;
        std::cout << "Number of nodes in results: " << cycles_map.size() << std::endl;
        auto cycles = cycles_map_to_cycles(cycles_map);        // main.cpp:542
        if (rank0) {
            {  // the cycles' labels in one device call (not a host copy of the whole graph)
                std::vector<uint64_t> nodes;
                for (const auto &[start, inner] : cycles_map)
                    for (const auto &c : inner) nodes.insert(nodes.end(), c.begin(), c.end());
                std::sort(nodes.begin(), nodes.end());
                nodes.erase(std::unique(nodes.begin(), nodes.end()), nodes.end());
                sdbg.PrefetchKeys(nodes);
            }
            const std::string out = settings.cycles_folder + "/cycles.txt";
            std::ofstream f(out);
            size_t idx = 0;
            for (const auto &[start, inner] : cycles_map)
                for (const auto &c : inner) {
                    f << ">cycle_" << idx++ << " start=" << start << " length=" << c.size() << "\n";
                    f << cycle_sequence(sdbg, c) << "\n";
                }
        }

        const double t_cycles_out = since(g_main_start);
        banner("🔸STEP 6: Finding relevant reads");             // main.cpp:544-551
        int n_files = 0;
        {
            std::istringstream iss(settings.input_files);
            std::string t;
            while (iss >> t) ++n_files;
        }
        const auto reads = run_and_debug_finding_of_relevant_reads(cycles, sdbg_build.reads(), sdbg,
                                                                   settings.gpus > 1 ? settings.mcomm : nullptr,
                                                                   std::max(1, n_files));
        if (settings.mcomm) {
            mcaat_comm_free(settings.mcomm);
            settings.mcomm = nullptr;
        }
        if (!rank0) return 0;  // rank 0 writes the outputs
        const double t_step6 = since(g_main_start);

        banner("🔸STEP 7: Order the spacers");                  // main.cpp:553-556
        const auto found_systems = run_and_debug_spacer_ordering(reads, sdbg, cycles, (unsigned)std::max<size_t>(1, settings.threads));

        const double t_step7 = since(g_main_start);
        if (settings.benchmark_file != "") {                   // main.cpp:559-569
            banner("🔸STEP 8: Compare to ground of truth using benchmark file");
            run_and_debug_benchmark_results(settings, found_systems);
        } else {
            banner("🔸STEP 8: Results");
            run_and_debug_results(found_systems);
        }
        std::cout << "══════════════════════════════════════════════" << std::endl;

        const double t_step8 = since(g_main_start);
        std::cout << "POST PROCESSING START:" << std::endl;    // main.cpp:573-581
        std::unordered_map<std::string, std::vector<std::string>> all_systems;
        for (const auto &[_sequence, repeat, spacers, _conf_a, _conf_b] : found_systems) all_systems[repeat] = spacers;
        CRISPRAnalyzer analyzer(all_systems, settings.output_file);
        analyzer.run_analysis();
        std::cout << "Saved in: " << settings.output_file << std::endl;

        try {                                                  // main.cpp:525,584-589: "<graph>/graph"
            fs::remove_all(settings.graph_folder + "/graph");
        } catch (const std::filesystem::filesystem_error &e) {
            std::cerr << "Warning: Could not remove graph folder: " << e.what() << std::endl;
        }
        if (ranks.watcher.joinable()) ranks.watcher.join();  // every rank ended cleanly
        {
            // where the rest of the wall goes (seconds since main; process start and exit are
            // outside): runtime init before the span, the span, cycles.txt, steps 6/7/8 and
            // CRISPRAnalyzer
            char line[320];
            snprintf(line, sizeof line,
                     "TIMING_TAIL init_s=%.6f span_end_s=%.6f cycles_out_s=%.6f step6_s=%.6f step7_s=%.6f "
                     "step8_s=%.6f analyzer_s=%.6f main_s=%.6f",
                     t_span_start, t_span_end, t_cycles_out - t_span_end, t_step6 - t_cycles_out,
                     t_step7 - t_step6, t_step8 - t_step7, since(g_main_start) - t_step8, since(g_main_start));
            std::cout << line << std::endl;
        }
        return 0;
    }
}
