// Factory templates (same names as hadoop-1.0.3/src/c++/pipes/api/hadoop/TemplateFactory.hh):
// TemplateFactory<Mapper, Reducer[, Partitioner[, Combiner[, RecordReader[, RecordWriter]]]]>.
#ifndef HBMR_TEMPLATE_FACTORY_HH
#define HBMR_TEMPLATE_FACTORY_HH

#include <type_traits>

#include "hadoop/Pipes.hh"

namespace HadoopPipes {

template <class M, class R, class P = void, class C = void, class RR = void, class RW = void>
class TemplateFactory : public Factory {
  template <class T, class Base, class Ctx>
  static Base* create(Ctx& ctx) {
    if constexpr (std::is_void<T>::value) {
      (void)ctx;
      return NULL;
    } else {
      return new T(ctx);
    }
  }

 public:
  Mapper* createMapper(MapContext& context) const override { return new M(context); }
  Reducer* createReducer(ReduceContext& context) const override { return new R(context); }
  Partitioner* createPartitioner(MapContext& context) const override {
    return create<P, Partitioner>(context);
  }
  Reducer* createCombiner(MapContext& context) const override {
    return create<C, Reducer>(context);
  }
  RecordReader* createRecordReader(MapContext& context) const override {
    return create<RR, RecordReader>(context);
  }
  RecordWriter* createRecordWriter(ReduceContext& context) const override {
    return create<RW, RecordWriter>(context);
  }
};

// Hadoop's numbered spellings.
template <class M, class R>
using TemplateFactory2 = TemplateFactory<M, R>;
template <class M, class R, class P>
using TemplateFactory3 = TemplateFactory<M, R, P>;
template <class M, class R, class P, class C>
using TemplateFactory4 = TemplateFactory<M, R, P, C>;
template <class M, class R, class P, class C, class RR>
using TemplateFactory5 = TemplateFactory<M, R, P, C, RR>;

}  // namespace HadoopPipes

#endif
