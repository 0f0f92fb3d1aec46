"""Uniform adapters over the oracle (CPU restatement) and the engine (HIP path via the C-ABI),
so that the transcribed reference tests run unchanged against both.

Canonical Subscribers form (string keyed, Go maps as dicts):
  {"subscriptions": {client: sub}, "shared": {filter: {client: sub}}, "inline": {id: sub}}
with sub = {"filter","identifier","qos","no_local","rap","rh","identifiers"}.
"""
import oracle as O


class OracleAdapter:
    name = "oracle"

    def __init__(self):
        self.x = O.OracleIndex()
        self._h = 0

    def subscribe(self, client, filter, qos=0, identifier=0, no_local=False, rap=False, rh=0):
        return self.x.subscribe(client, filter, qos, identifier, no_local, rap, rh)

    def unsubscribe(self, filter, client):
        return self.x.unsubscribe(filter, client)

    def inline_subscribe(self, filter, identifier):
        return self.x.inline_subscribe(filter, identifier)

    def inline_unsubscribe(self, identifier, filter):
        return self.x.inline_unsubscribe(identifier, filter)

    def retain_message(self, topic, payload=b"hello", retain=True, handle=None):
        if handle is None:
            self._h += 1
            handle = self._h
        return self.x.retain_message(topic, handle, len(payload), retain), handle

    def retained_delete(self, topic):
        self.x.retained_delete(topic)

    def retained_len(self):
        return self.x.retained_len()

    def subscribers(self, topic):
        s = self.x.subscribers(topic)
        s["inline"] = {int(k): v for k, v in s["inline"].items()}
        return s

    def messages(self, filter):
        return self.x.messages(filter)

    def path_exists(self, filter, d=0):
        return self.x.path_exists(filter, d)


def _sub_dict(s, with_idents=True):
    d = {"filter": s.filter, "identifier": s.identifier, "qos": s.qos, "no_local": s.no_local,
         "rap": s.retain_as_published, "rh": s.retain_handling}
    if with_idents:
        d["identifiers"] = None if s.identifiers is None else dict(s.identifiers)
    return d


def canonical(subs):
    """engine.Subscribers -> canonical dict (the oracle's JSON shape)."""
    return {
        "subscriptions": {c: _sub_dict(s) for c, s in subs.subscriptions.items()},
        "shared": {f: {c: _sub_dict(s) for c, s in m.items()} for f, m in subs.shared.items()},
        "inline": {i: {"filter": s.filter, "identifier": s.identifier, "qos": 0,
                       "no_local": False, "rap": False, "rh": 0}
                   for i, s in subs.inline_subscriptions.items()},
    }


class EngineAdapter:
    name = "engine"

    def __init__(self, fmt="spans", msg_image=True):
        from mqmatch import engine as E
        self.E = E
        self.x = E.TopicsIndex(0, fmt=fmt)
        if not msg_image:  # Messages by the particle walk instead of the level-order image
            self.x.engine.set_option(E.OPT_MSG_IMAGE, 0)
        self._h = 0

    def subscribe(self, client, filter, qos=0, identifier=0, no_local=False, rap=False, rh=0):
        return self.x.subscribe(client, self.E.Subscription(filter, identifier, qos, no_local, rap, rh))

    def unsubscribe(self, filter, client):
        return self.x.unsubscribe(filter, client)

    def inline_subscribe(self, filter, identifier):
        return self.x.inline_subscribe(self.E.InlineSubscription(filter, identifier))

    def inline_unsubscribe(self, identifier, filter):
        return self.x.inline_unsubscribe(identifier, filter)

    def retain_message(self, topic, payload=b"hello", retain=True, handle=None):
        if handle is None:
            self._h += 1
            handle = self._h
        r = self.x.engine.retain_message(topic, handle, len(payload), retain)
        return r, handle

    def retained_delete(self, topic):
        self.x.engine.retained_delete(topic)

    def retained_len(self):
        return self.x.engine.retained_len()

    def subscribers(self, topic):
        return canonical(self.x.subscribers(topic))

    def subscribers_batch(self, topics):
        return [canonical(s) for s in self.x.subscribers_batch(topics)]

    def messages(self, filter):
        return self.x.messages(filter)

    def messages_batch(self, filters):
        return self.x.messages_batch(filters)
