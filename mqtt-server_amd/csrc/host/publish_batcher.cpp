// Publish batching stage over the host TopicsIndex: header-only (publish_batcher.h); this unit
// instantiates the two batchers once for the library.
#include "publish_batcher.h"

namespace mq {
namespace host {

template class BasicBatcher<MapsPolicy>;
template class BasicBatcher<ViewsPolicy>;

}  // namespace host
}  // namespace mq
