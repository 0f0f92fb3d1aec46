"""mqmatch — MI355X topic-matching engine (host-side Python mirror of the Go TopicsIndex API)."""
