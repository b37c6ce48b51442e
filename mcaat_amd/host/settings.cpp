// settings.cpp — parse_arguments (reference src/main.cpp:89-301), same flags and errors.
#include <sys/sysinfo.h>

#include "settings.h"

namespace fs = std::filesystem;

double get_total_system_ram() {
    struct sysinfo mi;
    if (sysinfo(&mi) == 0) return (double)mi.totalram * mi.mem_unit / (1024.0 * 1024.0 * 1024.0);
    return 0.0;
}

static void print_help() {
    std::cout << "Usage: ./mcaat --input-files <file1> [file2] [options]\n"
              << "\nRequired:\n"
              << "  --input-files, -i <file1> [file2]  One or two input FASTA/FASTQ files (.gz, .bz2 ok)\n"
              << "\nOptional:\n"
              << "  --ram <amount>                  RAM to use (e.g., 4G, 500M). Default: 95% of system RAM\n"
              << "  --threads <num>                 Number of threads. Default: CPU cores - 2\n"
              << "  --output-folder <path>          Output directory. If not provided, a timestamped folder is created\n"
              << "  --benchmark <file>              File containing expected crispr sequences line separated\n"
              << "  --cycle-max-length <int>        Maximum cycle length to search (default in settings)\n"
              << "  --cycle-min-length <int>        Minimum cycle length to search (default in settings)\n"
              << "  --threshold-multiplicity <int>  Minimum multiplicity threshold for start nodes (default in settings)\n"
              << "  --low-abundance <true|false>    Enable low abundance mode for cycle filtering\n"
              << "  --settings <path>               Path to a key=value settings file (overridden by CLI args)\n"
              << "  --gpu <index>                   GPU to run the hot path on (default 0)\n"
              << "  --gpus <num>                    GPUs (one process each) sharing the run (default 1)\n"
              << "  --comm <rccl|shm>               Multi-GPU transport: RCCL over xGMI, or host shared memory\n"
              << "  --keep-graph                    Keep the graph as <graph folder>/graph.mcaat_sdbg (checkpoint)\n"
              << "  --load-graph <file>             Resume from a kept graph instead of building it\n"
              << "  --help, -h                      Show this help message\n";
}

Settings parse_arguments(int argc, char *argv[], bool create_dirs) {
    std::vector<std::string> input_files_default;
    Settings settings;
    const std::string timestamp = Settings::get_timestamp();

    // pre-scan for --settings (main.cpp:96-104)
    for (int j = 1; j < argc; ++j)
        if (std::string(argv[j]) == "--settings" && j + 1 < argc) {
            if (!settings.LoadFromFile(argv[j + 1]))
                throw std::runtime_error("Error: could not load settings from " + std::string(argv[j + 1]));
            break;
        }

    bool output_folder_provided = false, required_files_provided = false, input_files_from_settings = false;
    for (int i = 1; i < argc; ++i) {
        std::string arg = argv[i];
        if (arg == "--help" || arg == "-h" || arg.empty()) {
            print_help();
            exit(0);
        }
        if (arg == "--input-files" || arg == "-i") {
            while (++i < argc && argv[i][0] != '-') input_files_default.push_back(argv[i]);
            --i;
            required_files_provided = true;
        } else if (arg == "--benchmark") {
            if (++i < argc) settings.benchmark_file = argv[i];
            else throw std::runtime_error("Error: Missing value for --benchmark");
            --i;  // reference quirk (main.cpp:142): the value is re-read as a flag and ignored
        } else if (arg == "--ram") {
            if (++i >= argc) throw std::runtime_error("Error: Missing value for --ram");
            std::string ram_input = argv[i];
            try {
                if (!Settings::parse_ram(ram_input, settings.ram))
                    throw std::runtime_error("Error: Invalid RAM unit. Use B, K, M, or G.");
            } catch (const std::invalid_argument &) {
                throw std::runtime_error("Error: Invalid RAM value provided: " + ram_input);
            }
            const double total = get_total_system_ram();
            if (settings.ram < 1.0)
                throw std::runtime_error("Error: RAM value " + std::to_string(settings.ram) +
                                         " GB is too low (must be at least 1 GB)");
            if (settings.ram > total)
                throw std::runtime_error("Error: RAM value " + std::to_string(settings.ram) +
                                         " GB exceeds system total of " + std::to_string(total) + " GB");
        } else if (arg == "--threads") {
            if (++i < argc) settings.threads = std::stoul(argv[i]);
            else throw std::runtime_error("Error: Missing value for --threads");
        } else if (arg == "--output-folder" || arg == "--output_folder") {
            if (++i < argc) {
                settings.output_folder = argv[i];
                output_folder_provided = true;
            } else throw std::runtime_error("Error: Missing value for --output-folder");
        } else if (arg == "--cycle-max-length") {
            if (++i < argc) settings.cycle_finder_settings.cycle_max_length = std::stoi(argv[i]);
            else throw std::runtime_error("Error: Missing value for --cycle-max-length");
        } else if (arg == "--cycle-min-length") {
            if (++i < argc) settings.cycle_finder_settings.cycle_min_length = std::stoi(argv[i]);
            else throw std::runtime_error("Error: Missing value for --cycle-min-length");
        } else if (arg == "--threshold-multiplicity") {
            if (++i < argc) settings.cycle_finder_settings.threshold_multiplicity = std::stoull(argv[i]);
            else throw std::runtime_error("Error: Missing value for --threshold-multiplicity");
        } else if (arg == "--low-abundance") {
            if (++i >= argc) throw std::runtime_error("Error: Missing value for --low-abundance");
            std::string v = argv[i];
            std::transform(v.begin(), v.end(), v.begin(), ::tolower);
            settings.cycle_finder_settings.low_abundance = (v == "1" || v == "true" || v == "yes");
        } else if (arg == "--gpu") {
            if (++i < argc) settings.gpu = std::stoi(argv[i]);
            else throw std::runtime_error("Error: Missing value for --gpu");
        } else if (arg == "--gpus") {
            if (++i < argc) settings.gpus = std::stoi(argv[i]);
            else throw std::runtime_error("Error: Missing value for --gpus");
        } else if (arg == "--comm") {
            if (++i < argc) settings.comm = argv[i];
            else throw std::runtime_error("Error: Missing value for --comm");
        } else if (arg == "--keep-graph") {
            settings.keep_graph = true;
        } else if (arg == "--load-graph") {
            if (++i < argc) settings.load_graph = argv[i];
            else throw std::runtime_error("Error: Missing value for --load-graph");
        } else if (arg == "--settings") {
            ++i;  // handled in the pre-scan
        }
    }
    if (input_files_default.empty() && !settings.input_files.empty()) {
        std::istringstream iss(settings.input_files);
        std::string tok;
        while (iss >> tok) input_files_default.push_back(tok);
        required_files_provided = true;
        input_files_from_settings = true;
    }
    if (!required_files_provided && input_files_default.empty() && settings.input_files.empty())
        throw std::runtime_error("Error: No input files provided. Use --input-files <file1> [file2]");
    if (!output_folder_provided && settings.output_folder.empty()) settings.output_folder = "mcaat_run_" + timestamp;
    if (settings.graph_folder.empty()) settings.graph_folder = settings.output_folder + "/graph";
    if (settings.cycles_folder.empty()) settings.cycles_folder = settings.output_folder + "/cycles";
    if (settings.output_file.empty()) settings.output_file = settings.output_folder + "/CRISPR_Arrays.txt";

    std::cout << "Output folder: " << settings.output_folder << std::endl;
    std::cout << "Graph folder: " << settings.graph_folder << std::endl;
    std::cout << "Cycles folder: " << settings.cycles_folder << std::endl;
    std::cout << "CycleFinder settings: max_length=" << settings.cycle_finder_settings.cycle_max_length
              << " min_length=" << settings.cycle_finder_settings.cycle_min_length
              << " threshold_mult=" << settings.cycle_finder_settings.threshold_multiplicity
              << " low_abundance=" << (settings.cycle_finder_settings.low_abundance ? "true" : "false")
              << " threads=" << settings.threads << std::endl;
    if (create_dirs) {
        try {
            fs::create_directories(settings.output_folder);
            fs::create_directories(settings.graph_folder);
            fs::create_directories(settings.cycles_folder);
        } catch (const fs::filesystem_error &e) {
            throw std::runtime_error("Error: Could not create directories: " + std::string(e.what()));
        }
    }
    if (input_files_default.size() < 1 || input_files_default.size() > 2)
        throw std::runtime_error("Error: You must provide one or two input files.");
    for (const auto &file : input_files_default) {
        if (!fs::exists(file)) throw std::runtime_error("Error: Input file " + file + " does not exist.");
        if (required_files_provided && !input_files_from_settings) {
            if (!settings.input_files.empty()) settings.input_files += " ";
            settings.input_files += file;
        }
    }
    if (settings.gpus < 1 || settings.gpus > 64) throw std::runtime_error("Error: --gpus must be in [1, 64]");
    if (settings.comm != "rccl" && settings.comm != "shm") throw std::runtime_error("Error: --comm must be rccl or shm");
    if (settings.threads == 0) settings.threads = std::thread::hardware_concurrency() - 2;
    if (settings.ram == 0.0) settings.ram = get_total_system_ram() * 0.95;
    return settings;
}
