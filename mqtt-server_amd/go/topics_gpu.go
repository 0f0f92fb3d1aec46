//go:build mqmatch

// topics_gpu.go — reference-side binding of the MI355X engine (include/mqmatch.h).
//
// Drop this file (with go.mod's module github.com/xyzj/mqtt-server) next to topics.go and build
// with `-tags mqmatch` and CGO_ENABLED=1: it replaces the TopicsIndex of topics.go:349-698 with
// the same exported API, backed by the C-ABI. topics.go's TopicsIndex, NewTopicsIndex and the
// particle types must then be excluded from the build (`//go:build !mqmatch` on topics.go's
// index half); Subscribers, SelectShared, MergeSharedSelected, IsValidFilter, IsSharedFilter
// and the alias types stay as they are. No Go toolchain exists in the build container, so this
// file is not compiled there; parity is proven through the same C-ABI by tests/.
package mqtt

/*
#cgo CFLAGS: -I${SRCDIR}/mqmatch/include
#cgo LDFLAGS: -L${SRCDIR}/mqmatch/lib -lmqmatch -Wl,-rpath,${SRCDIR}/mqmatch/lib
#include <stdlib.h>
#include "mqmatch.h"
*/
import "C"

import (
	"fmt"
	"sync"
	"unsafe"

	"github.com/xyzj/mqtt-server/packets"
)

// interner maps strings to dense u32 ids and back (client IDs, full filter strings).
type interner struct {
	ids  map[string]uint32
	strs []string
}

func newInterner() *interner { return &interner{ids: map[string]uint32{}} }

func (n *interner) id(s string) uint32 {
	if v, ok := n.ids[s]; ok {
		return v
	}
	v := uint32(len(n.strs))
	n.ids[s] = v
	n.strs = append(n.strs, s)
	return v
}

type subKey struct {
	client uint32
	filter uint32
}

// TopicsIndex is the engine-backed index; same exported surface as topics.go:350-353.
type TopicsIndex struct {
	Retained *packets.Packets
	h        *C.mq_index
	mu       sync.Mutex // guards the interners and the stored-subscription tables
	clients  *interner
	filters  *interner
	topics   *interner // retained topic names: handle = topic id
	stored   map[subKey]packets.Subscription
	inline   map[int]InlineSubscription // by identifier, for rematerialising handlers
	inlineBy map[subKey]InlineSubscription
}

// NewTopicsIndex (topics.go:356-364).
func NewTopicsIndex() *TopicsIndex {
	var h *C.mq_index
	cfg := C.mq_config{device: 0}
	if rc := C.mq_index_create(&cfg, &h); rc < 0 {
		panic(fmt.Sprintf("mq_index_create: %d %s", rc, C.GoString(C.mq_last_error())))
	}
	return &TopicsIndex{
		Retained: packets.NewPackets(),
		h:        h,
		clients:  newInterner(),
		filters:  newInterner(),
		topics:   newInterner(),
		stored:   map[subKey]packets.Subscription{},
		inline:   map[int]InlineSubscription{},
		inlineBy: map[subKey]InlineSubscription{},
	}
}

func cstr(s string) (*C.char, C.uint32_t) {
	if len(s) == 0 {
		return nil, 0
	}
	return (*C.char)(unsafe.Pointer(unsafe.StringData(s))), C.uint32_t(len(s))
}

func must(rc C.int, what string) C.int {
	if rc < 0 {
		panic(fmt.Sprintf("%s: %d %s", what, rc, C.GoString(C.mq_last_error())))
	}
	return rc
}

// Subscribe (topics.go:401-419).
func (x *TopicsIndex) Subscribe(client string, sub packets.Subscription) bool {
	x.mu.Lock()
	defer x.mu.Unlock()
	cid, fid := x.clients.id(client), x.filters.id(sub.Filter)
	flags := C.uint8_t(0)
	if sub.NoLocal {
		flags |= C.MQ_SUB_NOLOCAL
	}
	if sub.RetainAsPublished {
		flags |= C.MQ_SUB_RAP
	}
	flags |= C.uint8_t(sub.RetainHandling&3) << C.MQ_SUB_RH_SHIFT
	p, n := cstr(sub.Filter)
	rc := must(C.mq_subscribe(x.h, p, n, C.uint32_t(cid), C.uint32_t(fid), C.uint8_t(sub.Qos), flags,
		C.int32_t(sub.Identifier)), "mq_subscribe")
	x.stored[subKey{cid, fid}] = sub
	return rc == 1
}

// Unsubscribe (topics.go:423-448).
func (x *TopicsIndex) Unsubscribe(filter, client string) bool {
	x.mu.Lock()
	defer x.mu.Unlock()
	p, n := cstr(filter)
	return must(C.mq_unsubscribe(x.h, p, n, C.uint32_t(x.clients.id(client))), "mq_unsubscribe") == 1
}

// InlineSubscribe (topics.go:368-378).
func (x *TopicsIndex) InlineSubscribe(sub InlineSubscription) bool {
	x.mu.Lock()
	defer x.mu.Unlock()
	fid := x.filters.id(sub.Filter)
	p, n := cstr(sub.Filter)
	rc := must(C.mq_inline_subscribe(x.h, p, n, C.int32_t(sub.Identifier), C.uint32_t(fid)), "mq_inline_subscribe")
	x.inlineBy[subKey{uint32(sub.Identifier), fid}] = sub
	return rc == 1
}

// InlineUnsubscribe (topics.go:382-397).
func (x *TopicsIndex) InlineUnsubscribe(id int, filter string) bool {
	x.mu.Lock()
	defer x.mu.Unlock()
	p, n := cstr(filter)
	return must(C.mq_inline_unsubscribe(x.h, p, n, C.int32_t(id)), "mq_inline_unsubscribe") == 1
}

// RetainMessage (topics.go:453-476). The Go packets map stays the store of packets; the
// engine keeps the retain paths and liveness and returns the same 1/0/-1.
func (x *TopicsIndex) RetainMessage(pk packets.Packet) int64 {
	x.mu.Lock()
	defer x.mu.Unlock()
	handle := uint64(x.topics.id(pk.TopicName))
	p, n := cstr(pk.TopicName)
	var out C.int64_t
	must(C.mq_retain_message(x.h, p, n, C.uint64_t(handle), C.uint32_t(len(pk.Payload)),
		boolU8(pk.FixedHeader.Retain), &out), "mq_retain_message")
	if len(pk.Payload) > 0 {
		x.Retained.Add(pk.TopicName, pk)
	} else {
		x.Retained.Delete(pk.TopicName)
	}
	return int64(out)
}

// RetainedDelete is what server.go:1726 calls instead of x.Retained.Delete in the expiry sweep,
// so the engine drops the entry but keeps the retain path (Q12).
func (x *TopicsIndex) RetainedDelete(topic string) {
	x.mu.Lock()
	defer x.mu.Unlock()
	p, n := cstr(topic)
	C.mq_retained_delete(x.h, p, n)
	x.Retained.Delete(topic)
}

func boolU8(b bool) C.uint8_t {
	if b {
		return 1
	}
	return 0
}

func pack(items []string) ([]byte, []uint64) {
	offs := make([]uint64, len(items)+1)
	total := 0
	for _, s := range items {
		total += len(s)
	}
	buf := make([]byte, 0, total+1)
	for i, s := range items {
		buf = append(buf, s...)
		offs[i+1] = uint64(len(buf))
	}
	if len(buf) == 0 {
		buf = append(buf, 0)
	}
	return buf, offs
}

// Messages (topics.go:525-527).
func (x *TopicsIndex) Messages(filter string) []packets.Packet {
	x.mu.Lock()
	defer x.mu.Unlock()
	buf, offs := pack([]string{filter})
	var r *C.mq_msg_result
	must(C.mq_messages_batch(x.h, (*C.uint8_t)(&buf[0]), (*C.uint64_t)(&offs[0]), 1, &r), "mq_messages_batch")
	defer C.mq_result_free(unsafe.Pointer(r))
	hs := unsafe.Slice((*uint64)(unsafe.Pointer(r.handles)), int(r.n_handles))
	pks := []packets.Packet{}
	for _, h := range hs {
		if pk, ok := x.Retained.Get(x.topics.strs[h]); ok {
			pks = append(pks, pk)
		}
	}
	return pks
}

// Subscribers (topics.go:583-590): a batch of one.
func (x *TopicsIndex) Subscribers(topic string) *Subscribers {
	return x.SubscribersBatch([]string{topic})[0]
}

// SubscribersBatch matches many topics in one engine call; the batching stage in
// publishToSubscribers (server.go:984-1021) feeds it.
func (x *TopicsIndex) SubscribersBatch(topics []string) []*Subscribers {
	x.mu.Lock()
	defer x.mu.Unlock()
	buf, offs := pack(topics)
	var r *C.mq_match_result
	must(C.mq_match_batch(x.h, (*C.uint8_t)(&buf[0]), (*C.uint64_t)(&offs[0]), C.uint32_t(len(topics)), &r),
		"mq_match_batch")
	defer C.mq_result_free(unsafe.Pointer(r))
	tr := unsafe.Slice(r.topics, int(r.n_topics))
	rows := unsafe.Slice(r.sub_rows, int(r.n_sub_rows))
	shared := unsafe.Slice(r.shared_rows, int(r.n_shared_rows))
	inl := unsafe.Slice(r.inline_rows, int(r.n_inline_rows))
	out := make([]*Subscribers, len(topics))
	for i := range topics {
		t := tr[i]
		s := &Subscribers{
			Shared:              map[string]map[string]packets.Subscription{},
			SharedSelected:      map[string]packets.Subscription{},
			Subscriptions:       map[string]packets.Subscription{},
			InlineSubscriptions: map[int]InlineSubscription{},
		}
		// rows in gather order: a client's client row precedes its ident rows
		for _, cr := range rows[t.sub_base : t.sub_base+C.uint64_t(t.sub_cap)] {
			switch cr.meta & C.MQ_ROW_KIND_MASK {
			case 0: // client row: the merged Subscription
				base := x.stored[subKey{uint32(cr.client_id), uint32(cr.filter_id)}]
				base.Qos = byte(cr.meta & C.MQ_META_QOS_MASK)
				base.NoLocal = cr.meta&C.MQ_META_NOLOCAL != 0
				base.Identifiers = map[string]int{base.Filter: base.Identifier}
				s.Subscriptions[x.clients.strs[cr.client_id]] = base
			case C.MQ_ROW_IDENT: // a further Identifiers entry of that client
				sub := s.Subscriptions[x.clients.strs[cr.client_id]]
				sub.Identifiers[x.filters.strs[cr.filter_id]] = int(cr.identifier)
			}
		}
		for _, sr := range shared[t.shared_base : t.shared_base+C.uint64_t(t.n_shared)] {
			f, c := x.filters.strs[sr.filter_id], x.clients.strs[sr.client_id]
			if _, ok := s.Shared[f]; !ok {
				s.Shared[f] = map[string]packets.Subscription{}
			}
			s.Shared[f][c] = x.stored[subKey{uint32(sr.client_id), uint32(sr.filter_id)}]
		}
		for _, lr := range inl[t.inline_base : t.inline_base+C.uint64_t(t.n_inline)] {
			s.InlineSubscriptions[int(lr.identifier)] = x.inlineBy[subKey{uint32(lr.identifier), uint32(lr.filter_id)}]
		}
		out[i] = s
	}
	return out
}
