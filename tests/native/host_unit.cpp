// Host-only unit tests of the native runtime (CLI grammar, MT19937, report formats, stats, JSON,
// count parsing). Built twice: plainly (`make unit`) and under ASan+UBSan (`make asan`).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "mireduce/cli.hpp"
#include "mireduce/fault.hpp"
#include "mireduce/mt19937.hpp"
#include "mireduce/peer_access.hpp"
#include "mireduce/report.hpp"
#include "mireduce/timer.hpp"
#include "mireduce/types.hpp"

using namespace mireduce;

static int g_fail = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

static void test_peer_plan() {
  // bandwidth_test --peer: ordered pairs, no self pairs, row-major; matrix table shape
  CHECK(peer_pairs(0).empty() && peer_pairs(1).empty());
  const auto p2 = peer_pairs(2);
  CHECK(p2.size() == 2 && p2[0] == std::make_pair(0, 1) && p2[1] == std::make_pair(1, 0));
  const auto p8 = peer_pairs(8);
  CHECK(p8.size() == 56);
  for (auto [s, d] : p8) CHECK(s != d && s >= 0 && d < 8);
  std::vector<double> v(9, 0.0);
  v[1] = 12.5;
  v[3] = 99.0;
  const std::string t = peer_matrix(3, v, "GB/s");
  CHECK(t.find("12.5") != std::string::npos && t.find("99.0") != std::string::npos);
  CHECK(t.find("(GB/s)") != std::string::npos);
  int lines = 0;
  for (char c : t) lines += c == '\n';
  CHECK(lines == 5);  // title, column header, 3 source rows
}

static void test_cli() {
  const char* argv[] = {"prog", "--method=SUM", "-type=double", "--cpufinal", "-n=16M", "--list=a,b,,c", "--neg=-5"};
  CmdArgs a(7, argv);
  std::string s;
  CHECK(a.program() == "prog");
  CHECK(a.get_str("method", &s) && s == "SUM");
  CHECK(a.get_str("type", &s) && s == "double");
  CHECK(a.has("cpufinal") && !a.get_str("cpufinal", &s));
  uint64_t n = 0;
  CHECK(a.get_uint("n", &n) && n == (16ull << 20));
  std::vector<std::string> l;
  CHECK(a.get_list("list", &l) && l.size() == 3 && l[2] == "c");
  int64_t v = 0;
  CHECK(a.get_int("neg", &v) && v == -5);
  CHECK(a.unknown({"method", "type", "cpufinal", "n", "list"}).size() == 1);
  bool threw = false;
  try {
    const char* bad[] = {"prog", "method=SUM"};
    CmdArgs b(2, bad);
  } catch (const CliError&) {
    threw = true;
  }
  CHECK(threw);
  threw = false;
  try {
    const char* bad[] = {"prog", "--n=12x"};
    CmdArgs b(2, bad);
    uint64_t x;
    b.get_uint("n", &x);
  } catch (const CliError&) {
    threw = true;
  }
  CHECK(threw);
  uint64_t c = 0;
  CHECK(parse_count("1e9", &c) && c == 1000000000ull);
  CHECK(parse_count("4k", &c) && c == 4096);
  CHECK(parse_count("2G", &c) && c == (2ull << 30));
  CHECK(!parse_count("abc", &c) && !parse_count("1.5e0", &c));
}

static void test_types() {
  DType t;
  Op o;
  CHECK(parse_dtype("DOUBLE", &t) && t == DType::Float64);
  CHECK(parse_dtype("Int", &t) && t == DType::Int32);
  CHECK(parse_dtype("int64", &t) && t == DType::Int64);
  CHECK(!parse_dtype("char", &t));
  CHECK(parse_op_strict("SUM", &o) && o == Op::Sum);
  CHECK(!parse_op_strict("sum", &o));
  CHECK(parse_op("max", &o) && o == Op::Max);
  CHECK(default_acc(DType::Int32, Op::Sum) == DType::Int64);
  CHECK(default_acc(DType::Float32, Op::Min) == DType::Float32);
  CHECK(std::string(dtype_gnuplot_name(DType::Float64)) == "DOUBLE");
}

static void test_mt() {
  Mt19937 g;
  const uint64_t key[4] = {0x123, 0x234, 0x345, 0x456};
  g.init_by_array(key, 4);
  const uint32_t expect[5] = {1067595299u, 955945823u, 477289528u, 4107218783u, 4228976476u};
  for (uint32_t e : expect) CHECK(g.genrand_int32() == e);
  Mt19937 h(5489u);
  CHECK(h.genrand_int32() == 3499211612u);  // std::mt19937 default-seed first output
}

static void test_report() {
  CHECK(gnuplot_header() == "# DATATYPE OP NODES GB/sec");
  CHECK(gnuplot_line("INT", "SUM", 1024, 146.684) == "INT SUM 1024    146.684");
  CHECK(throughput_line(92.7729, 0.00072, 16777216, 1, 256) ==
        "Reduction, Throughput = 92.7729 GB/s, Time = 0.00072 s, Size = 16777216 Elements, NumDevsUsed = 1, Workgroup = 256");
  Stats s = compute_stats({3, 1, 2, 4});
  CHECK(s.count == 4 && s.min == 1 && s.max == 4 && s.median == 2.5 && std::fabs(s.mean - 2.5) < 1e-12);
  Json j;
  j.set("a", "x\"y").set("b", 1.5).set("c", static_cast<int64_t>(-3)).set("d", true).set("e", std::vector<double>{1, 2});
  CHECK(j.str() == "{\"a\": \"x\\\"y\", \"b\": 1.5, \"c\": -3, \"d\": true, \"e\": [1,2]}");
  StopWatch w;
  w.start();
  w.stop();
  w.start();
  w.stop();
  CHECK(w.sessions() == 2 && w.laps_ms().size() == 2 && w.average_ms() >= 0);
}

static void test_fault_spec() {
  FaultSpec f = parse_fault_spec("");
  CHECK(f.kind == FaultSpec::Kind::None);
  f = parse_fault_spec("exit");
  CHECK(f.kind == FaultSpec::Kind::Exit && f.rank == 1 && f.step == 0);
  f = parse_fault_spec("hang@3:17");
  CHECK(f.kind == FaultSpec::Kind::Hang && f.rank == 3 && f.step == 17);
  f = parse_fault_spec("delay=250@0:2");
  CHECK(f.kind == FaultSpec::Kind::Delay && f.delay_ms == 250 && f.rank == 0 && f.step == 2);
  f = parse_fault_spec("corrupt:5");
  CHECK(f.kind == FaultSpec::Kind::Corrupt && f.rank == 1 && f.step == 5);
  for (const char* bad : {"boom", "exit@", "exit@x", "hang:-1", "delay=", "corrupt@1:2x"}) {
    bool threw = false;
    try {
      parse_fault_spec(bad);
    } catch (const std::invalid_argument&) {
      threw = true;
    }
    CHECK(threw);
  }
  FaultInjector inj(parse_fault_spec("corrupt@2:4"));
  CHECK(!inj.at(1, 4, "unit") && !inj.at(2, 3, "unit"));
  CHECK(inj.at(2, 4, "unit"));
  CHECK(!inj.at(2, 4, "unit"));  // fires once
  FaultInjector d(parse_fault_spec("delay=1@0:0"));
  CHECK(!d.at(0, 0, "unit"));
}

static void test_peer_verdict() {
  // the native twin of parallel/topology.py peer_verdict
  auto yes = [](int, int) { return true; };
  auto no = [](int, int) { return false; };
  const std::vector<PeerKey> node = {{"h", "g0", 0}, {"h", "g1", 1}, {"h", "g2", 2}};
  for (int me = 0; me < 3; ++me) CHECK(peer_verdict(node, me, yes).empty());
  CHECK(peer_verdict(node, 1, no) == "device 1 cannot access peer device 0 (rank 0)");
  // a one-way link: 0 can map 2 but 2 cannot map 0 -> only rank 2 objects
  auto oneway = [](int a, int b) { return !(a == 2 && b == 0); };
  CHECK(peer_verdict(node, 0, oneway).empty());
  CHECK(peer_verdict(node, 2, oneway).find("cannot access peer device 0") != std::string::npos);
  // ranks sharing one physical GPU need no peer access (one-GPU rehearsals)
  const std::vector<PeerKey> shared = {{"h", "g0", 0}, {"h", "g0", 0}, {"h", "g0", 0}};
  CHECK(peer_verdict(shared, 2, no).empty());
  // another host: IPC handles do not cross hosts
  const std::vector<PeerKey> two_hosts = {{"a", "g0", 0}, {"b", "g0", 0}};
  CHECK(peer_verdict(two_hosts, 0, yes).find("runs on host b") != std::string::npos);
  // same index, different GPU (e.g. different visibility masks)
  const std::vector<PeerKey> alias = {{"h", "g0", 0}, {"h", "g7", 0}};
  CHECK(peer_verdict(alias, 1, yes).find("a different GPU") != std::string::npos);
  CHECK(peer_verdict(node, 5, yes) == "rank index out of range");
  // agreement: identical text on every rank, failing ranks only, in rank order
  CHECK(agree_verdicts({"", "", ""}).empty());
  CHECK(agree_verdicts({"", "x", "", "y"}) == "rank 1: x; rank 3: y");
  // the injected fault kind parses and is not a step fault
  FaultInjector f(parse_fault_spec("nopeer@1"));
  CHECK(f.no_peer(1) && !f.no_peer(0) && !f.at(1, 0, "unit"));
}

int main() {
  test_peer_verdict();
  test_cli();
  test_peer_plan();
  test_fault_spec();
  test_types();
  test_mt();
  test_report();
  if (g_fail) {
    std::fprintf(stderr, "host_unit: %d failures\n", g_fail);
    return 1;
  }
  std::printf("host_unit: all checks passed\n");
  return 0;
}
