"""Synthetic RFQ corpus: emails, formal RFQ documents and line-item tables.

Used by the benchmark (docs/s on synthetic RFQ documents, BASELINE.json), the
tokenizer trainer and the tests.  The length distribution follows the
reference's recorded workload: prompts of 262-958 tokens with the
current template ≈ 465 tokens of shared prefix plus 0.26 tokens/char of document
text, i.e. documents of roughly 300-2,400 characters (p50 ≈ 900).  Everything is
deterministic in the seed.
"""
from __future__ import annotations

import random
from dataclasses import dataclass, field

FIRST = ["rajesh", "anita", "li wei", "maria", "john", "sofia", "ahmed", "yuki", "carlos",
         "priya", "tom", "elena", "kwame", "sara", "dmitri", "fatima", "lukas", "mei", "omar",
         "grace", "arjun", "chloe", "ivan", "nadia"]
LAST = ["sharma", "gupta", "chen", "garcia", "smith", "rossi", "khan", "tanaka", "lopez",
        "patel", "brown", "novak", "mensah", "cohen", "petrov", "haddad", "weber", "wong",
        "nasser", "kim", "iyer", "martin", "ivanov", "ali"]
COMPANY_A = ["subha", "apex", "nova", "delta", "orion", "vertex", "quantum", "stellar", "zenith",
             "titan", "pioneer", "summit", "atlas", "fusion", "crest", "harbor", "everest",
             "polaris", "sigma", "matrix"]
COMPANY_B = ["tek electros", "industries", "components ltd", "automation gmbh", "systems inc",
             "engineering co", "electronics pvt ltd", "manufacturing llc", "technologies",
             "precision works", "controls sa", "power solutions", "devices corp"]
SUPPLIERS = ["amphenol", "te connectivity", "molex", "digikey", "mouser", "arrow", "avnet",
             "rs components", "farnell", "würth elektronik", "phoenix contact", "harting"]
CITIES = ["chennai", "pune", "bengaluru", "shenzhen", "munich", "rotterdam", "austin", "detroit",
          "singapore", "dubai", "milan", "osaka", "são paulo", "toronto", "lyon", "gdansk"]
ITEMS = [("Circular connector 8 pin - bayonet", "62GB-56T-16-8S"),
         ("SMA-SMA cable 1.5m", "ACX9016"), ("RJ45 jack w/ gasket + panel lock", "RJFTV7G"),
         ("USB-C receptacle, shielded, 16 pin", "114017"), ("M12 sensor cable 5m", "M12-5A-PUR"),
         ("Terminal block 2.5mm2 grey", "UT2.5-GY"), ("Heat shrink 6mm black (1m)", "HS6-BK"),
         ("Toroidal transformer 230/24V 100VA", "TT-100-24"), ("Fuse holder 5x20 panel mount", "FH520"),
         ("Ethernet patch cord Cat6 2m", "C6-PC-2M"), ("DIN rail 35mm x 1m", "DIN35-1000"),
         ("Relay 24VDC DPDT 10A", "RL24-DPDT"), ("Ceramic capacitor 100nF 50V 0603", "CC0603-104"),
         ("Resistor 10k 1% 0805", "RC0805-10K"), ("Aluminium enclosure IP67 120x80", "AL-IP67-128"),
         ("Cable gland PG9 nylon", "CG-PG9"), ("Ferrite bead 600R 0805", "FB0805-600"),
         ("LED indicator 8mm green 24V", "LED8-GN-24"), ("Proximity sensor M18 PNP", "PS18-PNP"),
         ("Push button 22mm red", "PB22-RD"), ("Power supply 24V 5A DIN", "PSU24-5"),
         ("Stepper motor NEMA17 1.8deg", "NEMA17-18"), ("Copper busbar 20x5mm 1m", "CB205-1"),
         ("Coaxial connector N-type female", "N-F-BH")]
CURRENCIES = [("$", "{}"), ("USD", "{} USD"), ("€", "€{}"), ("EUR", "{} EUR"), ("£", "£{}"),
              ("₹", "₹{}"), ("rs", "{} rs"), ("euros", "{} euros"), ("dollars", "{} dollars"),
              ("GBP", "{} GBP"), ("INR", "INR {}")]
DOCS = ["ISO 9001 certificate", "RoHS declaration", "REACH compliance statement", "datasheet",
        "test report", "certificate of conformity", "material safety data sheet",
        "country of origin certificate", "warranty terms", "packing list"]
MONTHS = ["jan", "feb", "mar", "apr", "may", "jun", "jul", "aug", "sep", "oct", "nov", "dec"]


@dataclass
class LineItem:
    part_number: str
    description: str
    quantity: int
    target_price: float | None
    currency: str | None


@dataclass
class RFQDoc:
    text: str
    client_name: str
    client_email: str
    client_contact: str
    client_phone: str
    rfq_to: str
    delivery_location: str
    items: list[LineItem] = field(default_factory=list)


def _date(r: random.Random) -> str:
    d, m = r.randint(1, 28), r.choice(MONTHS)
    return r.choice([f"{d}-{m}", f"{m} {d}", f"{d:02d}/{MONTHS.index(m) + 1:02d}/2025",
                     f"end of {m}", f"2025-{MONTHS.index(m) + 1:02d}-{d:02d}"])


def make_rfq(seed: int, n_items: int | None = None, style: str | None = None) -> RFQDoc:
    r = random.Random(seed)
    contact = f"{r.choice(FIRST)} {r.choice(LAST)}"
    company = f"{r.choice(COMPANY_A)}{r.choice(['', ' '])}{r.choice(COMPANY_B)}"
    dom = company.split()[0].replace(" ", "") + r.choice([".net", ".com", ".in", ".de", ".co.uk"])
    email = r.choice(["sourcing", "purchase", "procurement", contact.split()[0]]) + "@" + dom
    phone = r.choice(["+91-9{0}-{1}", "+1 ({0}) {1}", "+49 {0} {1}", "+86 {0}-{1}"]).format(
        r.randint(1000, 9999), r.randint(10000, 99999))
    supplier = r.choice(SUPPLIERS)
    city = r.choice(CITIES)
    n = n_items if n_items is not None else r.choice([1, 2, 3, 3, 4, 4, 5, 6, 8, 10, 14])
    items = []
    for _ in range(n):
        desc, pn = r.choice(ITEMS)
        if r.random() < 0.5:
            pn = f"{pn}-{r.randint(10, 99)}"
        qty = r.choice([5, 10, 25, 50, 100, 250, 300, 400, 500, 750, 1000, 2500, 5000])
        price = None if r.random() < 0.2 else round(r.uniform(0.05, 900), r.choice([0, 2]))
        cur = r.choice(CURRENCIES) if price is not None else None
        items.append(LineItem(pn, desc, qty, price, cur[0] if cur else None))
    style = style or r.choice(["informal", "formal", "table", "terse"])
    due, deliv = _date(r), _date(r)
    docs = r.sample(DOCS, r.randint(0, 3))
    lines = []
    if style == "informal":
        lines.append(f"hello {supplier},")
        lines.append(f"pls send ur best prices for below. shipment to {city} by {deliv} is needed.")
        for it in items:
            lines.append(f"- part no: {it.part_number}")
            lines.append(r.choice([f"qty: {it.quantity}", f"need {it.quantity}pcs",
                                   f"Qty = {it.quantity:,}"]))
            lines.append(f"desc: {it.description}")
            if it.target_price is not None:
                fmt = dict(CURRENCIES)[it.currency]
                lines.append(r.choice(["target: ", "tp: ", "around "]) + fmt.format(it.target_price)
                             + r.choice(["", "/pc", " per unit", " is acceptable"]))
        if docs:
            lines.append("also share " + ", ".join(docs) + ".")
        lines.append(r.choice(["note: lead times are critical, share alt parts if quicker.",
                               "quote validity min 30 days pls.", ""]))
        lines += ["thx,", contact, company, email, phone]
    elif style == "formal":
        lines.append(f"REQUEST FOR QUOTATION No. RFQ-{r.randint(1000, 99999)}")
        lines.append(f"Date: {_date(r)}")
        lines.append(f"To: {supplier.title()} Sales Department")
        lines.append(f"From: {company.title()}, Procurement")
        lines.append("")
        lines.append("Dear Sir/Madam,")
        lines.append(f"We kindly request your quotation for the items listed below, to be delivered "
                     f"to our facility in {city.title()} no later than {deliv}. Please submit "
                     f"your offer by {due}.")
        for i, it in enumerate(items, 1):
            price = ""
            if it.target_price is not None:
                price = " | Target price: " + dict(CURRENCIES)[it.currency].format(it.target_price)
            lines.append(f"{i}. {it.description} | P/N {it.part_number} | Quantity: "
                         f"{it.quantity}{price}")
        if docs:
            lines.append("Required documents: " + "; ".join(docs) + ".")
        lines.append("Payment terms: 60 days net. Incoterms: DAP.")
        lines += ["Best regards,", contact.title(), "Purchasing Manager", company.title(),
                  f"Email: {email}", f"Phone: {phone}"]
    elif style == "table":
        lines.append(f"Hi {supplier.title()} team,")
        lines.append(f"Please quote the following. Delivery: {city.title()}, required by {deliv}.")
        lines.append("| # | Part Number | Description | Qty | Target Price |")
        lines.append("|---|---|---|---|---|")
        for i, it in enumerate(items, 1):
            tp = dict(CURRENCIES)[it.currency].format(it.target_price) if it.target_price is not None else "-"
            lines.append(f"| {i} | {it.part_number} | {it.description} | {it.quantity} | {tp} |")
        lines.append(f"Quote needed by {due}.")
        lines += ["Regards,", f"{contact.title()} ({company.title()})", email, phone]
    else:
        lines.append(f"RFQ - {company}")
        for it in items:
            tp = dict(CURRENCIES)[it.currency].format(it.target_price) if it.target_price is not None else ""
            lines.append(f"{it.part_number} x{it.quantity} {tp}".strip())
        lines.append(f"ship {city}, {deliv}. {contact}, {email}")
    return RFQDoc("\n".join(lines), company, email, contact, phone, supplier, city, items)


TERMS = [
    "Prices shall be quoted firm and fixed for the validity period stated in the offer and "
    "shall include packing suitable for sea and road freight.",
    "All goods shall be supplied new, of current manufacture, and traceable to the original "
    "component manufacturer by lot and date code.",
    "Partial shipments are acceptable only with prior written approval of the purchasing "
    "department; each shipment shall carry the purchase order number on every package.",
    "The supplier shall state the country of origin and the HS tariff code of every line "
    "item together with the unit net weight.",
    "Lead times shall be given in calendar days from receipt of the purchase order; "
    "deviations from the requested delivery schedule shall be highlighted.",
    "Alternative or equivalent parts may be offered only if clearly marked as alternates "
    "with the full manufacturer part number and a datasheet link.",
    "Quality documentation, including certificates of conformity and test reports, shall "
    "accompany each delivery or be sent electronically before dispatch.",
    "Warranty shall cover a minimum period of twenty-four months from the date of delivery "
    "against defects in material and workmanship.",
    "Invoices shall reference the purchase order and line numbers; payment terms are sixty "
    "days net from receipt of a correct invoice.",
    "The buyer reserves the right to award the order in whole or in part, or to reject any "
    "offer without stating reasons.",
]


def make_long_rfq(seed: int, min_chars: int = 9000) -> RFQDoc:
    """A multi-page formal RFQ whose text runs past the reference's 8,000-character
    input cap (rfq_agent.py:147-149): letterhead, a long numbered item list and the
    buyer's terms and conditions -- BASELINE config 4's "multi-page PDF RFQs
    (prefill-heavy)".  Rendered as a PDF (docgen.rfq_attachment) it spans 4-5 pages;
    the parsed text is truncated to 8,000 characters by the prompt builder, i.e. a
    prompt of ~2.9 K tokens on the in-tree tokenizer (~2.4 K after the shared prefix)."""
    base = make_rfq(seed, n_items=0, style="formal")
    r = random.Random(seed * 7 + 1)
    head = base.text.splitlines()[:7]
    tail = base.text.splitlines()[7:]
    items, lines = [], list(head)
    lines.append("Section 1 - Items to be quoted")
    i = 0
    while True:
        desc, pn = r.choice(ITEMS)
        pn = f"{pn}-{r.randint(10, 99)}" if r.random() < 0.6 else pn
        qty = r.choice([10, 25, 50, 100, 250, 500, 1000, 2500])
        price = None if r.random() < 0.3 else round(r.uniform(0.05, 900), 2)
        cur = r.choice(CURRENCIES) if price is not None else None
        items.append(LineItem(pn, desc, qty, price, cur[0] if cur else None))
        i += 1
        tp = (" | Target price: " + dict(CURRENCIES)[cur[0]].format(price)) if price is not None else ""
        lines.append(f"{i}. {desc} | P/N {pn} | Quantity: {qty} pcs | Delivery: "
                     f"{_date(r)}{tp}")
        if i >= 40 or len("\n".join(lines)) > min_chars * 0.6:
            break
    lines.append("Section 2 - Terms and conditions")
    for k, t in enumerate(TERMS * 3, 1):
        lines.append(f"2.{k} {t}")
        if len("\n".join(lines + tail)) > min_chars:
            break
    lines.append("Section 3 - Required documents")
    lines.append("; ".join(r.sample(DOCS, 4)) + ".")
    lines += tail
    return RFQDoc("\n".join(lines), base.client_name, base.client_email, base.client_contact,
                  base.client_phone, base.rfq_to, base.delivery_location, items)


def corpus(n: int, seed: int = 0) -> list[RFQDoc]:
    return [make_rfq(seed * 1_000_003 + i) for i in range(n)]


def reference_like_completion(doc: RFQDoc, seed: int = 0) -> str:
    """A plausible extraction JSON for `doc` (tokenizer corpus / golden shapes)."""
    import json

    r = random.Random(seed)
    obj = {
        "title": doc.text.splitlines()[0][:60], "client_name": doc.client_name,
        "client_email": doc.client_email, "client_contact": doc.client_contact,
        "client_phone": doc.client_phone, "rfq_to": doc.rfq_to,
        "delivery_location": doc.delivery_location, "delivery_deadline": None,
        "response_due_date": None, "description": "Request for quotation",
        "line_items": [dict(part_number=i.part_number, description=i.description,
                            quantity=i.quantity, target_price=i.target_price,
                            currency=i.currency) for i in doc.items],
        "requested_documents": [], "confidence_score": round(r.uniform(0.6, 0.95), 2),
        "missing_fields": ["response_due_date"], "requires_review": r.random() < 0.3,
    }
    return json.dumps(obj, ensure_ascii=False, indent=r.choice([None, 2]))


def decode_hints(doc: RFQDoc) -> dict:
    """Bench-only decoding hints for a synthetic document (SamplingParams keywords).

    Random-init weights carry no knowledge of when an extraction is complete, so the
    benchmark shapes each constrained decode like the document's extraction: the
    grammar's SYNTHETIC profile (string / array caps, schema-typed values only) and
    one ``line_items`` object per part the document mentions.  The service never
    applies these (it decodes with the REFERENCE profile)."""
    from ..engine.grammar import PROFILE_SYNTHETIC
    from ..service.hints import estimate_line_items

    return {"min_items": estimate_line_items(doc.text), "profile": PROFILE_SYNTHETIC}
