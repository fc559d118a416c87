"""Random window-engine queries shared by the GPU parity tests and the CPU
hipRTC code-generation tests."""


def window_case(rng):
    """Random `every e1=S[f1] -> e2=S[f2] within W` over one stream (window engine)."""
    f1 = rng.choice(["price > {c}f", "x < {c}", "volume >= {c}L", "price > 10.0 and x != {c}",
                     "x % 3 == 1", "price * 2.0f > {c}f"]).format(c=rng.randint(0, 20))
    f2 = rng.choice(["price > e1.price", "x <= e1.x", "sym == e1.sym and price < e1.price",
                     "price > e1.price * 1.05", "x < e1.x + {c}", "volume != e1.volume and x > e1.x",
                     "price + 1.0f > e1.price", "(x / 2) > e1.x"]).format(c=rng.randint(0, 5))
    w = rng.choice([0, 1, 5, 40, 1000])
    partitioned = rng.random() < 0.7
    sel = ["e1.sym as a", "e1.price as b", "e2.price as c", "e2.volume as d", "e1.x as e"]
    if rng.random() < 0.3:
        sel.append("e2.x * 2 as f")
    q = (f"@info(name = 'query1') from every e1=S[{f1}] -> e2=S[{f2}] within {w} milliseconds "
         f"select {', '.join(sel)} insert into Out;")
    defs = "define stream S (sym string, price float, volume long, x int); "
    app = defs + (f"partition with (sym of S) begin {q} end;" if partitioned else q)
    return app, partitioned
