//go:build mqmatch

// topics_gpu.go — reference-side binding of the MI355X engine (include/mqmatch.h).
//
// Drop this file (with go.mod's module github.com/xyzj/mqtt-server) next to topics.go and build
// with `-tags mqmatch` and CGO_ENABLED=1: it replaces the TopicsIndex of topics.go:349-698 with
// the same exported API, backed by the C-ABI. topics.go's TopicsIndex, NewTopicsIndex and the
// particle types must then be excluded from the build (`//go:build !mqmatch` on topics.go's
// index half); Subscribers, SelectShared, MergeSharedSelected, IsValidFilter, IsSharedFilter
// and the alias types stay as they are. server.go is unchanged: TopicsIndex.Retained keeps the
// method set server.go uses (Add, Get, GetAll, Len, Delete — server.go:980, 1717-1726), and
// its Add / Delete reach the engine. No Go toolchain exists in the build container, so this
// file is not compiled there; the same C-ABI calls, locking and id recycling are exercised by
// the C++ host mirror (csrc/host/topics_index.cpp, tests/cpp/test_topics_index.cpp).
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
	"math"
	"strings"
	"sync"
	"time"
	"unsafe"

	"github.com/xyzj/mqtt-server/packets"
)

// noClient is an id no subscription uses: Unsubscribe for a client the index never saw still
// answers whether the filter's particle exists (topics.go:434-437).
const noClient = math.MaxUint32

// epochs tracks the match batches in flight. A batch's results may name any id that was in use
// when it began, so an id released at time r is reused only once every batch begun before r
// has ended.
type epochs struct {
	mu     sync.Mutex
	clock  uint64
	active map[uint64]int
}

func (e *epochs) begin() uint64 {
	e.mu.Lock()
	defer e.mu.Unlock()
	e.clock++
	e.active[e.clock]++
	return e.clock
}

func (e *epochs) end(t uint64) {
	e.mu.Lock()
	defer e.mu.Unlock()
	if e.active[t]--; e.active[t] == 0 {
		delete(e.active, t)
	}
}

func (e *epochs) now() uint64 {
	e.mu.Lock()
	defer e.mu.Unlock()
	e.clock++
	return e.clock
}

func (e *epochs) oldest() uint64 {
	e.mu.Lock()
	defer e.mu.Unlock()
	m := uint64(math.MaxUint64)
	for t := range e.active {
		if t < m {
			m = t
		}
	}
	return m
}

// idTable maps strings (client IDs, filters, retained topics) to dense u32 ids, referenced by
// what uses them; an unreferenced id is released and later reused (epochs). Guarded by
// TopicsIndex.tables.
type idTable struct {
	ep   *epochs
	ids  map[string]uint32
	strs []string
	refs []uint32
	free []freeID // oldest release first
}

type freeID struct {
	id uint32
	at uint64
}

func newIDTable(ep *epochs) *idTable { return &idTable{ep: ep, ids: map[string]uint32{}} }

// intern returns the id of s, creating it unreferenced if new.
func (t *idTable) intern(s string) uint32 {
	if v, ok := t.ids[s]; ok {
		return v
	}
	var v uint32
	if len(t.free) > 0 && t.free[0].at < t.ep.oldest() {
		v = t.free[0].id
		t.free = t.free[1:]
		t.strs[v] = s
	} else {
		if len(t.strs) == noClient {
			panic("mqmatch: id space exhausted")
		}
		v = uint32(len(t.strs))
		t.strs = append(t.strs, s)
		t.refs = append(t.refs, 0)
	}
	t.ids[s] = v
	return v
}

func (t *idTable) find(s string) (uint32, bool) {
	v, ok := t.ids[s]
	return v, ok
}

func (t *idTable) ref(id uint32) { t.refs[id]++ }

// unref drops a reference; at zero the id is released at time `now`. tidy releases an id that
// was interned but never referenced.
func (t *idTable) unref(id uint32, now uint64) {
	t.refs[id]--
	t.tidy(id, now)
}

func (t *idTable) tidy(id uint32, now uint64) {
	if t.refs[id] != 0 {
		return
	}
	if v, ok := t.ids[t.strs[id]]; !ok || v != id {
		return // already released
	}
	delete(t.ids, t.strs[id]) // t.strs[id] stays readable for batches still in flight
	t.free = append(t.free, freeID{id, now})
}

type subKey struct {
	client uint32
	filter uint32
}

// RetainedPackets is TopicsIndex.Retained (topics.go:351): the reference's packets.Packets
// store, which server.go reads and sweeps directly (server.go:980, 1717-1726), wrapped so that
// entries added or deleted outside RetainMessage reach the engine as well — the expiry sweep's
// Delete drops the engine's entry and keeps the retain path (Q12); an Add makes the entry live
// again.
type RetainedPackets struct {
	*packets.Packets
	x *TopicsIndex
}

// Add (packets/packets.go:79-83).
func (r *RetainedPackets) Add(id string, val packets.Packet) {
	x := r.x
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.Lock()
	h := x.topics.intern(id)
	x.tables.Unlock()
	p, n := cstr(id)
	must(C.mq_retained_set(x.h, p, n, C.uint64_t(h), C.uint32_t(len(val.Payload)), boolU8(val.FixedHeader.Retain)),
		"mq_retained_set")
	x.mapAdd(id, h, val)
}

// Delete (packets/packets.go:113-117).
func (r *RetainedPackets) Delete(id string) {
	x := r.x
	x.upd.Lock()
	defer x.upd.Unlock()
	p, n := cstr(id)
	must(C.mq_retained_delete(x.h, p, n), "mq_retained_delete")
	x.mapDelete(id)
}

// TopicsIndex is the engine-backed index; same exported surface as topics.go:350-353.
//
// Locking: updates are serialised by upd (the engine serialises them as well); readers
// (Subscribers, Messages) never take it, so a GPU round trip never waits for an update's lock
// nor an update for a match. tables guards the id tables and the stored subscriptions.
type TopicsIndex struct {
	Retained *RetainedPackets
	h        *C.mq_index
	upd      sync.Mutex
	tables   sync.RWMutex
	ep       *epochs
	// the batching stage Subscribers goes through (started on first use)
	batcherOnce sync.Once
	batcher     *MatchBatcher
	clients  *idTable
	filters  *idTable
	topics   *idTable // retained topic names: handle = topic id, referenced while in Retained
	stored   map[subKey]packets.Subscription
	inlineBy map[subKey]InlineSubscription // (identifier, filter)
}

// NewTopicsIndex (topics.go:356-364).
func NewTopicsIndex() *TopicsIndex {
	var h *C.mq_index
	cfg := C.mq_config{device: 0}
	if rc := C.mq_index_create(&cfg, &h); rc < 0 {
		panic(fmt.Sprintf("mq_index_create: %d %s", rc, C.GoString(C.mq_last_error())))
	}
	ep := &epochs{active: map[uint64]int{}}
	x := &TopicsIndex{
		h:        h,
		ep:       ep,
		clients:  newIDTable(ep),
		filters:  newIDTable(ep),
		topics:   newIDTable(ep),
		stored:   map[subKey]packets.Subscription{},
		inlineBy: map[subKey]InlineSubscription{},
	}
	x.Retained = &RetainedPackets{Packets: packets.NewPackets(), x: x}
	return x
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

func boolU8(b bool) C.uint8_t {
	if b {
		return 1
	}
	return 0
}

// Subscribe (topics.go:401-419).
func (x *TopicsIndex) Subscribe(client string, sub packets.Subscription) bool {
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.Lock()
	cid, fid := x.clients.intern(client), x.filters.intern(sub.Filter)
	x.tables.Unlock()
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
	x.tables.Lock()
	k := subKey{cid, fid}
	if _, ok := x.stored[k]; !ok {
		x.clients.ref(cid)
		x.filters.ref(fid)
	}
	x.stored[k] = sub
	x.tables.Unlock()
	return rc == 1
}

// Unsubscribe (topics.go:423-448). An unknown client is looked up, never interned.
func (x *TopicsIndex) Unsubscribe(filter, client string) bool {
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.RLock()
	cid, okc := x.clients.find(client)
	fid, okf := x.filters.find(filter)
	x.tables.RUnlock()
	c := uint32(noClient)
	if okc {
		c = cid
	}
	p, n := cstr(filter)
	rc := must(C.mq_unsubscribe(x.h, p, n, C.uint32_t(c)), "mq_unsubscribe")
	if okc && okf {
		x.tables.Lock()
		k := subKey{cid, fid}
		if _, ok := x.stored[k]; ok {
			delete(x.stored, k)
			now := x.ep.now()
			x.clients.unref(cid, now)
			x.filters.unref(fid, now)
		}
		x.tables.Unlock()
	}
	return rc == 1
}

// InlineSubscribe (topics.go:368-378).
func (x *TopicsIndex) InlineSubscribe(sub InlineSubscription) bool {
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.Lock()
	fid := x.filters.intern(sub.Filter)
	x.tables.Unlock()
	p, n := cstr(sub.Filter)
	rc := must(C.mq_inline_subscribe(x.h, p, n, C.int32_t(sub.Identifier), C.uint32_t(fid)), "mq_inline_subscribe")
	x.tables.Lock()
	k := subKey{uint32(sub.Identifier), fid}
	if _, ok := x.inlineBy[k]; !ok {
		x.filters.ref(fid)
	}
	x.inlineBy[k] = sub
	x.tables.Unlock()
	return rc == 1
}

// InlineUnsubscribe (topics.go:382-397).
func (x *TopicsIndex) InlineUnsubscribe(id int, filter string) bool {
	x.upd.Lock()
	defer x.upd.Unlock()
	p, n := cstr(filter)
	rc := must(C.mq_inline_unsubscribe(x.h, p, n, C.int32_t(id)), "mq_inline_unsubscribe")
	x.tables.Lock()
	if fid, ok := x.filters.find(filter); ok {
		k := subKey{uint32(id), fid}
		if _, ok := x.inlineBy[k]; ok {
			delete(x.inlineBy, k)
			x.filters.unref(fid, x.ep.now())
		}
	}
	x.tables.Unlock()
	return rc == 1
}

// mapAdd / mapDelete keep the packet store and the topic id's reference together (upd held).
func (x *TopicsIndex) mapAdd(topic string, h uint32, pk packets.Packet) {
	if _, ok := x.Retained.Packets.Get(topic); !ok {
		x.tables.Lock()
		x.topics.ref(h)
		x.tables.Unlock()
	}
	x.Retained.Packets.Add(topic, pk)
}

func (x *TopicsIndex) mapDelete(topic string) {
	_, live := x.Retained.Packets.Get(topic)
	x.Retained.Packets.Delete(topic)
	x.tables.Lock()
	if h, ok := x.topics.find(topic); ok {
		if live {
			x.topics.unref(h, x.ep.now())
		} else {
			x.topics.tidy(h, x.ep.now())
		}
	}
	x.tables.Unlock()
}

// RetainMessage (topics.go:453-476). The Go packets map stays the store of packets and answers
// the -1 case from the replaced packet as the reference does; the engine keeps the retain paths
// and liveness.
func (x *TopicsIndex) RetainMessage(pk packets.Packet) int64 {
	x.upd.Lock()
	defer x.upd.Unlock()
	x.tables.Lock()
	h := x.topics.intern(pk.TopicName)
	x.tables.Unlock()
	p, n := cstr(pk.TopicName)
	var out C.int64_t
	must(C.mq_retain_message(x.h, p, n, C.uint64_t(h), C.uint32_t(len(pk.Payload)),
		boolU8(pk.FixedHeader.Retain), &out), "mq_retain_message")
	if len(pk.Payload) > 0 {
		x.mapAdd(pk.TopicName, h, pk)
		return 1
	}
	var r int64
	if pke, ok := x.Retained.Packets.Get(pk.TopicName); ok && len(pke.Payload) > 0 && pke.FixedHeader.Retain {
		r = -1
	}
	x.mapDelete(pk.TopicName)
	return r
}

// pack concatenates strings for the engine: offsets, plus the 16 readable padding bytes the
// C-ABI asks of an input buffer (include/mqmatch.h).
func pack(items []string) ([]byte, []uint64) {
	offs := make([]uint64, len(items)+1)
	total := 0
	for _, s := range items {
		total += len(s)
	}
	buf := make([]byte, 0, total+16)
	for i, s := range items {
		buf = append(buf, s...)
		offs[i+1] = uint64(len(buf))
	}
	buf = append(buf, make([]byte, 16)...)
	return buf, offs
}

// Messages (topics.go:525-579). A filter without wildcards is the packet store's own lookup,
// as in the reference (topics.go:539-544); the others run on the engine.
func (x *TopicsIndex) Messages(filter string) []packets.Packet {
	pks := []packets.Packet{}
	if len(filter) == 0 || x.Retained.Len() == 0 {
		return pks
	}
	if !strings.ContainsRune(filter, '#') && !strings.ContainsRune(filter, '+') {
		if pk, ok := x.Retained.Get(filter); ok {
			pks = append(pks, pk)
		}
		return pks
	}
	stamp := x.ep.begin()
	defer x.ep.end(stamp)
	buf, offs := pack([]string{filter})
	var r *C.mq_msg_result
	must(C.mq_messages_batch(x.h, (*C.uint8_t)(&buf[0]), (*C.uint64_t)(&offs[0]), 1, &r), "mq_messages_batch")
	hs := unsafe.Slice((*uint64)(unsafe.Pointer(r.handles)), int(r.n_handles))
	topics := make([]string, len(hs))
	x.tables.RLock()
	for i, h := range hs {
		topics[i] = x.topics.strs[h]
	}
	x.tables.RUnlock()
	C.mq_result_free(unsafe.Pointer(r))
	for _, t := range topics {
		if pk, ok := x.Retained.Get(t); ok {
			pks = append(pks, pk)
		}
	}
	return pks
}

// Subscribers (topics.go:583-590). publishToSubscribers calls it once per publish from every
// connection goroutine (server.go:1000); the call goes through the index's batching stage, which
// matches the topics of many goroutines with one engine call (MatchBatcher below), so server.go
// keeps calling Subscribers unchanged.
func (x *TopicsIndex) Subscribers(topic string) *Subscribers {
	x.batcherOnce.Do(func() { x.batcher = NewMatchBatcher(x, DefaultMaxBatch, DefaultMinFill, DefaultMaxDelay) })
	return x.batcher.Subscribers(topic)
}

// The batching stage's defaults (SURVEY.md §8f.1; DESIGN.md §7 has the measured batch latency).
const (
	DefaultMaxBatch = 16384                  // topics per engine call at most
	DefaultMinFill  = 1024                   // a batch with fewer topics waits for more ...
	DefaultMaxDelay = 200 * time.Microsecond // ... up to this long
)

// MatchBatcher is the batching stage of the publish pipeline (SURVEY.md §8f.1): connection
// goroutines hand their topic to one loop goroutine per index and wait for their result; the loop
// takes every request queued when the previous batch is done — under load, what arrived while it
// was matched — waits up to maxDelay for more when it holds fewer than minFill, and matches the
// batch with one SubscribersBatch call (one cgo call). Each caller gets exactly Subscribers(topic)
// on the index state the batch ran against (readers take no root lock in the reference either,
// topics.go:583, Q11), so the OnSelectSubscribers hook (hooks.go:360-367), SelectShared /
// MergeSharedSelected and the fan-out after it (server.go:1001-1021) are unchanged.
type MatchBatcher struct {
	x        *TopicsIndex
	in       chan matchReq
	maxBatch int
	minFill  int
	maxDelay time.Duration
	done     chan struct{}
}

type matchReq struct {
	topic string
	reply chan *Subscribers
}

var replyChans = sync.Pool{New: func() any { return make(chan *Subscribers, 1) }}

// NewMatchBatcher starts a batching stage over x.
func NewMatchBatcher(x *TopicsIndex, maxBatch, minFill int, maxDelay time.Duration) *MatchBatcher {
	if maxBatch <= 0 {
		maxBatch = DefaultMaxBatch
	}
	if minFill <= 0 || minFill > maxBatch {
		minFill = maxBatch
	}
	b := &MatchBatcher{x: x, in: make(chan matchReq, 4*maxBatch), maxBatch: maxBatch, minFill: minFill,
		maxDelay: maxDelay, done: make(chan struct{})}
	go b.loop()
	return b
}

// Subscribers enqueues topic and waits for the batch it joins.
func (b *MatchBatcher) Subscribers(topic string) *Subscribers {
	r := replyChans.Get().(chan *Subscribers)
	b.in <- matchReq{topic, r}
	s := <-r
	replyChans.Put(r)
	return s
}

// Close matches what is queued and stops the loop; no Subscribers call may follow.
func (b *MatchBatcher) Close() {
	close(b.in)
	<-b.done
}

func (b *MatchBatcher) loop() {
	defer close(b.done)
	batch := make([]matchReq, 0, b.maxBatch)
	topics := make([]string, 0, b.maxBatch)
	timer := time.NewTimer(time.Hour)
	timer.Stop()
	for {
		r, ok := <-b.in
		if !ok {
			return
		}
		batch = append(batch[:0], r)
		open := true
	drain: // everything queued now, without waiting
		for len(batch) < b.maxBatch {
			select {
			case r, ok := <-b.in:
				if !ok {
					open = false
					break drain
				}
				batch = append(batch, r)
			default:
				break drain
			}
		}
		if open && len(batch) < b.minFill && b.maxDelay > 0 { // a small batch waits a little for more
			timer.Reset(b.maxDelay)
		wait:
			for len(batch) < b.maxBatch {
				select {
				case r, ok := <-b.in:
					if !ok {
						break wait
					}
					batch = append(batch, r)
					if len(batch) >= b.minFill {
						break wait
					}
				case <-timer.C:
					break wait
				}
			}
			timer.Stop()
		}
		topics = topics[:0]
		for _, r := range batch {
			topics = append(topics, r.topic)
		}
		for i, s := range b.x.SubscribersBatch(topics) {
			batch[i].reply <- s
		}
		clear(batch) // drop the references to the replies
	}
}

// SubscribersBatch matches many topics in one engine call (span format: the index's own
// records plus patches, per topic or shared by a merge set, include/mqmatch.h); the batching stage in
// publishToSubscribers (server.go:984-1021) feeds it. A subscription removed between the match
// and the rebuild below is rebuilt from its record.
func (x *TopicsIndex) SubscribersBatch(topics []string) []*Subscribers {
	stamp := x.ep.begin()
	defer x.ep.end(stamp)
	buf, offs := pack(topics)
	var r *C.mq_span_result
	must(C.mq_match_spans(x.h, (*C.uint8_t)(&buf[0]), (*C.uint64_t)(&offs[0]), C.uint32_t(len(topics)), &r),
		"mq_match_spans")
	defer C.mq_result_free(unsafe.Pointer(r)) // after the tables' read lock below is released
	ts := unsafe.Slice(r.topics, int(r.n_topics))
	spans := unsafe.Slice(r.spans, int(r.n_spans))
	patches := unsafe.Slice(r.patches, int(r.n_patches))
	// merge-set patches (MQ_TOPIC_SET_PATCHES): row x<<MQ_SET_ROW_BITS|k is record k of the
	// topic's x-th may-merge particle, whose first row is merge_rows[merge_row_base[topic]+x]
	setPatches := unsafe.Slice(r.set_patches, int(r.n_set_patches))
	mergeRows := unsafe.Slice(r.merge_rows, int(r.n_merge_rows))
	var mergeBase []C.uint32_t
	if r.merge_row_base != nil {
		mergeBase = unsafe.Slice(r.merge_row_base, int(r.n_topics))
	}
	const rowBits = uint32(C.MQ_SET_ROW_BITS)
	inl := unsafe.Slice(r.inline_rows, int(r.n_inline_rows))
	picked := unsafe.Slice(r.picked_rows, int(r.n_picked_rows))
	subPool := unsafe.Slice(r.sub_pool, int(r.sub_pool_len))
	shrPool := unsafe.Slice(r.shared_pool, int(r.shared_pool_len))
	pickedOnly := r.flags&C.MQ_SPANS_PICKED != 0

	x.tables.RLock()
	defer x.tables.RUnlock()
	stored := func(c, f uint32, ident int32, meta uint32) packets.Subscription {
		if s, ok := x.stored[subKey{c, f}]; ok {
			return s
		}
		return packets.Subscription{Filter: x.filters.strs[f], Identifier: int(ident), Qos: byte(meta & C.MQ_META_QOS_MASK)}
	}
	out := make([]*Subscribers, len(topics))
	patched := map[uint32]uint32{} // topic row -> meta
	for i := range topics {
		t := ts[i]
		s := &Subscribers{
			Shared:              map[string]map[string]packets.Subscription{},
			SharedSelected:      map[string]packets.Subscription{},
			Subscriptions:       map[string]packets.Subscription{},
			InlineSubscriptions: map[int]InlineSubscription{},
		}
		clear(patched)
		if t.flags&C.MQ_TOPIC_SET_PATCHES != 0 {
			mr := mergeRows[mergeBase[i]:]
			for _, pt := range setPatches[t.patch_base : t.patch_base+C.uint64_t(t.n_patches)] {
				row := uint32(pt.row)
				patched[uint32(mr[row>>rowBits])+row&(1<<rowBits-1)] = uint32(pt.meta)
			}
		} else {
			for _, pt := range patches[t.patch_base : t.patch_base+C.uint64_t(t.n_patches)] {
				patched[uint32(pt.row)] = uint32(pt.meta)
			}
		}
		addShared := func(sr C.mq_shared_row) {
			f, c := x.filters.strs[sr.filter_id], x.clients.strs[sr.client_id]
			if _, ok := s.Shared[f]; !ok {
				s.Shared[f] = map[string]packets.Subscription{}
			}
			s.Shared[f][c] = stored(uint32(sr.client_id), uint32(sr.filter_id), 0, 0)
		}
		// records in gather order: a client's client row precedes its ident rows
		row := uint32(0)
		for _, sp := range spans[t.span_base : t.span_base+C.uint64_t(t.n_spans)] {
			for _, cr := range subPool[sp.sub_off : sp.sub_off+sp.n_sub] {
				meta := uint32(cr.meta)
				if m, ok := patched[row]; ok {
					meta = m
				}
				row++
				switch meta & C.MQ_ROW_KIND_MASK {
				case 0: // client row: the merged Subscription
					base := stored(uint32(cr.client_id), uint32(cr.filter_id), int32(cr.identifier), meta)
					base.Qos = byte(meta & C.MQ_META_QOS_MASK)
					base.NoLocal = meta&C.MQ_META_NOLOCAL != 0
					base.Identifiers = map[string]int{base.Filter: base.Identifier}
					s.Subscriptions[x.clients.strs[cr.client_id]] = base
				case C.MQ_ROW_IDENT: // a further Identifiers entry of that client
					sub := s.Subscriptions[x.clients.strs[cr.client_id]]
					sub.Identifiers[x.filters.strs[cr.filter_id]] = int(cr.identifier)
				}
			}
			if !pickedOnly {
				for _, sr := range shrPool[sp.shr_off : sp.shr_off+sp.n_shr] {
					addShared(sr)
				}
			}
		}
		if pickedOnly {
			for _, sr := range picked[t.picked_base : t.picked_base+C.uint64_t(t.n_shared)] {
				addShared(sr)
			}
		}
		for _, lr := range inl[t.inline_base : t.inline_base+C.uint64_t(t.n_inline)] {
			in, ok := x.inlineBy[subKey{uint32(lr.identifier), uint32(lr.filter_id)}]
			if !ok { // unsubscribed since the match
				in = InlineSubscription{Subscription: packets.Subscription{Filter: x.filters.strs[lr.filter_id],
					Identifier: int(lr.identifier)}}
			}
			s.InlineSubscriptions[int(lr.identifier)] = in
		}
		out[i] = s
	}
	return out
}
