// Pipes WordCount with a C++ partitioner (cf. src/examples/pipes/impl/wordcount-part.cc):
// words are routed by their first byte.
#include <string>

#include "hadoop/Pipes.hh"
#include "hadoop/StringUtils.hh"
#include "hadoop/TemplateFactory.hh"

class Map : public HadoopPipes::Mapper {
 public:
  explicit Map(HadoopPipes::TaskContext&) {}
  void map(HadoopPipes::MapContext& ctx) override {
    for (const std::string& w : HadoopUtils::splitString(ctx.getInputValue(), " "))
      if (!w.empty()) ctx.emit(w, "1");
  }
};

class Reduce : public HadoopPipes::Reducer {
 public:
  explicit Reduce(HadoopPipes::TaskContext&) {}
  void reduce(HadoopPipes::ReduceContext& ctx) override {
    int sum = 0;
    while (ctx.nextValue()) sum += HadoopUtils::toInt(ctx.getInputValue());
    ctx.emit(ctx.getInputKey(), HadoopUtils::toString(sum));
  }
};

class FirstBytePartitioner : public HadoopPipes::Partitioner {
 public:
  explicit FirstBytePartitioner(HadoopPipes::TaskContext&) {}
  int partition(const std::string& key, int numOfReduces) override {
    return key.empty() ? 0 : (unsigned char)key[0] % numOfReduces;
  }
};

int main(int argc, char* argv[]) {
  HadoopPipes::setProgramArgs(argc, argv);
  return HadoopPipes::runTask(
             HadoopPipes::TemplateFactory<Map, Reduce, FirstBytePartitioner>()) ? 0 : 1;
}
