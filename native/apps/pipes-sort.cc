// Identity map/reduce over raw records (cf. src/examples/pipes/impl/sort.cc and
// the gridmix "pipesort" benchmark): the framework's shuffle does the sorting.
#include "hadoop/Pipes.hh"
#include "hadoop/TemplateFactory.hh"

class Map : public HadoopPipes::Mapper {
 public:
  explicit Map(HadoopPipes::TaskContext&) {}
  void map(HadoopPipes::MapContext& ctx) override {
    ctx.emit(ctx.getInputKey(), ctx.getInputValue());
  }
};

class Reduce : public HadoopPipes::Reducer {
 public:
  explicit Reduce(HadoopPipes::TaskContext&) {}
  void reduce(HadoopPipes::ReduceContext& ctx) override {
    while (ctx.nextValue()) ctx.emit(ctx.getInputKey(), ctx.getInputValue());
  }
};

int main(int argc, char* argv[]) {
  HadoopPipes::setProgramArgs(argc, argv);
  return HadoopPipes::runTask(HadoopPipes::TemplateFactory<Map, Reduce>()) ? 0 : 1;
}
