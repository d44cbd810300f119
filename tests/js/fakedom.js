// A minimal DOM for node-level tests of the web apps' DOM wiring (no jsdom on this image): an HTML
// parser for the markup the pages and kf.js generate, elements with attributes / dataset / classList,
// form-control properties (value, checked, disabled, hidden, selected options), the selector subset
// the pages use (tag, #id, .class, [attr], [attr=v], :checked, descendant and comma groups),
// closest / matches, bubbling events with on<type> handlers, and <dialog> showModal / close.
"use strict";

const VOID = new Set(["input", "br", "img", "meta", "link", "hr", "col", "source", "wbr"]);
const ENT = { amp: "&", lt: "<", gt: ">", quot: '"', "#39": "'", apos: "'", times: "×", nbsp: " " };
const decode = (s) => s.replace(/&(#\d+|#x[0-9a-f]+|[a-z]+);/gi, (m, e) =>
  e[0] === "#" ? String.fromCharCode(e[1] === "x" ? parseInt(e.slice(2), 16) : parseInt(e.slice(1), 10)) : (e in ENT ? ENT[e] : m));
const enc = (s) => String(s).replace(/&/g, "&amp;").replace(/</g, "&lt;").replace(/>/g, "&gt;").replace(/"/g, "&quot;");

class Node {
  constructor() { this.parentNode = null; this.childNodes = []; }
  get parentElement() { return this.parentNode instanceof Element ? this.parentNode : null; }
  remove() { if (this.parentNode) this.parentNode.removeChild(this); }
}

class Text extends Node {
  constructor(t) { super(); this.nodeType = 3; this.data = t; }
  get textContent() { return this.data; }
  set textContent(v) { this.data = String(v); }
  serialize() { return enc(this.data); }
}

class ClassList {
  constructor(el) { this.el = el; }
  _get() { return (this.el.getAttribute("class") || "").split(/\s+/).filter(Boolean); }
  contains(c) { return this._get().includes(c); }
  add(...cs) { this.el.setAttribute("class", [...new Set([...this._get(), ...cs])].join(" ")); }
  remove(...cs) { this.el.setAttribute("class", this._get().filter((c) => !cs.includes(c)).join(" ")); }
  toggle(c, force) {
    const on = force === undefined ? !this.contains(c) : force;
    if (on) this.add(c); else this.remove(c);
    return on;
  }
}

class Element extends Node {
  constructor(tag, ownerDocument) {
    super();
    this.nodeType = 1;
    this.tagName = tag.toUpperCase();
    this.localName = tag.toLowerCase();
    this.attributes = {};
    this.listeners = {};
    this.style = {};
    this.ownerDocument = ownerDocument;
    this.classList = new ClassList(this);
    this._value = undefined;
    this._checked = undefined;
    this.open = false;
  }
  // ---- attributes ----
  getAttribute(n) { return Object.prototype.hasOwnProperty.call(this.attributes, n) ? this.attributes[n] : null; }
  setAttribute(n, v) { this.attributes[n] = String(v); }
  hasAttribute(n) { return Object.prototype.hasOwnProperty.call(this.attributes, n); }
  removeAttribute(n) { delete this.attributes[n]; }
  get id() { return this.getAttribute("id") || ""; }
  set id(v) { this.setAttribute("id", v); }
  get className() { return this.getAttribute("class") || ""; }
  set className(v) { this.setAttribute("class", v); }
  get dataset() {
    const out = {};
    for (const [k, v] of Object.entries(this.attributes))
      if (k.startsWith("data-")) out[k.slice(5).replace(/-([a-z])/g, (m, c) => c.toUpperCase())] = v;
    return out;
  }
  get name() { return this.getAttribute("name") || ""; }
  get type() { return (this.getAttribute("type") || (this.localName === "select" ? "select-one" : "text")).toLowerCase(); }
  // ---- form-control state ----
  get hidden() { return this.hasAttribute("hidden"); }
  set hidden(v) { if (v) this.setAttribute("hidden", ""); else this.removeAttribute("hidden"); }
  get disabled() { return this.hasAttribute("disabled"); }
  set disabled(v) { if (v) this.setAttribute("disabled", ""); else this.removeAttribute("disabled"); }
  get checked() { return this._checked === undefined ? this.hasAttribute("checked") : this._checked; }
  set checked(v) {
    this._checked = !!v;
    if (v && this.type === "radio" && this.name) {
      for (const r of this.ownerDocument.querySelectorAll(`input[name="${this.name}"]`)) if (r !== this) r._checked = false;
    }
  }
  get selected() { return this._selected === undefined ? this.hasAttribute("selected") : this._selected; }
  set selected(v) { this._selected = !!v; }
  get options() { return this.querySelectorAll("option"); }
  get value() {
    if (this.localName === "select") {
      const opts = this.options;
      const sel = opts.find((o) => o.selected) || opts[0];
      return sel ? sel.value : "";
    }
    if (this.localName === "option") return this.hasAttribute("value") ? this.getAttribute("value") : this.textContent.trim();
    if (this._value !== undefined) return this._value;
    if (this.localName === "textarea") return this.textContent;
    const v = this.getAttribute("value");
    return v !== null ? v : ((this.type === "checkbox" || this.type === "radio") ? "on" : "");
  }
  set value(v) {
    if (this.localName === "select") {
      for (const o of this.options) o._selected = o.value === String(v);
      return;
    }
    this._value = String(v);
  }
  // ---- tree ----
  get children() { return this.childNodes.filter((n) => n instanceof Element); }
  get firstChild() { return this.childNodes[0] || null; }
  appendChild(n) {
    if (n.parentNode) n.parentNode.removeChild(n);
    n.parentNode = this;
    this.childNodes.push(n);
    return n;
  }
  append(...ns) { ns.forEach((n) => this.appendChild(typeof n === "string" ? new Text(n) : n)); }
  removeChild(n) {
    const i = this.childNodes.indexOf(n);
    if (i >= 0) this.childNodes.splice(i, 1);
    n.parentNode = null;
    return n;
  }
  get textContent() { return this.childNodes.map((n) => n.textContent).join(""); }
  set textContent(v) { this.childNodes = []; if (v !== "" && v != null) this.appendChild(new Text(String(v))); }
  get innerHTML() { return this.childNodes.map((n) => n.serialize()).join(""); }
  set innerHTML(html) {
    this.childNodes.forEach((n) => { n.parentNode = null; });
    this.childNodes = [];
    parseInto(this, String(html), this.ownerDocument);
  }
  serialize() {
    const attrs = Object.entries(this.attributes).map(([k, v]) => (v === "" ? ` ${k}` : ` ${k}="${enc(v)}"`)).join("");
    if (VOID.has(this.localName)) return `<${this.localName}${attrs}>`;
    return `<${this.localName}${attrs}>${this.innerHTML}</${this.localName}>`;
  }
  // ---- selectors ----
  matches(sel) { return sel.split(",").some((s) => matchComplex(this, s.trim())); }
  closest(sel) {
    for (let e = this; e instanceof Element; e = e.parentNode) if (e.matches(sel)) return e;
    return null;
  }
  querySelectorAll(sel) {
    const out = [];
    const walk = (n) => {
      for (const c of n.childNodes) {
        if (c instanceof Element) {
          if (c.matches(sel)) out.push(c);
          walk(c);
        }
      }
    };
    walk(this);
    return out;
  }
  querySelector(sel) { return this.querySelectorAll(sel)[0] || null; }
  getElementsByTagName(t) { return this.querySelectorAll(t); }
  // ---- events ----
  addEventListener(type, fn) { (this.listeners[type] = this.listeners[type] || []).push(fn); }
  removeEventListener(type, fn) { this.listeners[type] = (this.listeners[type] || []).filter((f) => f !== fn); }
  dispatchEvent(ev) {
    ev.target = ev.target || this;
    ev.defaultPrevented = false;
    ev.preventDefault = () => { ev.defaultPrevented = true; };
    let stopped = false;
    ev.stopPropagation = () => { stopped = true; };
    for (let n = this; n && !stopped; n = ev.bubbles === false ? null : n.parentNode) {
      ev.currentTarget = n;
      const h = n["on" + ev.type];
      if (typeof h === "function") h.call(n, ev);
      for (const f of [...((n.listeners || {})[ev.type] || [])]) f.call(n, ev);
      if (n.ownerDocument && n === n.ownerDocument.documentElement) {
        for (const f of [...(n.ownerDocument.listeners[ev.type] || [])]) f.call(n.ownerDocument, ev);
      }
    }
    return !ev.defaultPrevented;
  }
  click() {
    if (this.disabled) return;
    if (this.type === "checkbox") this.checked = !this.checked;
    if (this.type === "radio") this.checked = true;
    this.dispatchEvent({ type: "click" });
    // a submit button submits its form
    if (this.localName === "button" && (this.getAttribute("type") || "submit") === "submit") {
      const form = this.closest("form");
      if (form) form.dispatchEvent({ type: "submit", submitter: this });
    }
  }
  focus() {}
  // ---- dialog ----
  showModal() { this.open = true; this.setAttribute("open", ""); }
  show() { this.showModal(); }
  close(v) {
    this.open = false;
    this.removeAttribute("open");
    if (v !== undefined) this.returnValue = v;
    this.dispatchEvent({ type: "close", bubbles: false });
  }
  get scrollHeight() { return 0; }
}

// ---- selector matching --------------------------------------------------------------------------------
function parseCompound(s) {
  const parts = { tag: null, id: null, classes: [], attrs: [], pseudo: [] };
  const re = /([a-zA-Z][\w-]*)|#([\w-]+)|\.([\w-]+)|\[([\w-]+)(?:([~|^$*]?=)(?:"([^"]*)"|'([^']*)'|([^\]]*)))?\]|:([\w-]+)/g;
  let m;
  let pos = 0;
  while ((m = re.exec(s)) !== null) {
    if (m.index !== pos) throw new Error(`fakedom: unsupported selector ${s}`);
    pos = re.lastIndex;
    if (m[1]) parts.tag = m[1].toLowerCase();
    else if (m[2]) parts.id = m[2];
    else if (m[3]) parts.classes.push(m[3]);
    else if (m[4]) parts.attrs.push([m[4], m[5], m[6] !== undefined ? m[6] : m[7] !== undefined ? m[7] : m[8]]);
    else if (m[9]) parts.pseudo.push(m[9]);
  }
  if (pos !== s.length) throw new Error(`fakedom: unsupported selector ${s}`);
  return parts;
}
function matchCompound(el, s) {
  const p = parseCompound(s);
  if (p.tag && p.tag !== "*" && el.localName !== p.tag) return false;
  if (p.id && el.id !== p.id) return false;
  if (p.classes.some((c) => !el.classList.contains(c))) return false;
  for (const [n, op, v] of p.attrs) {
    if (!el.hasAttribute(n)) return false;
    if (op === "=" && el.getAttribute(n) !== v) return false;
  }
  for (const ps of p.pseudo) {
    if (ps === "checked" && !(el.checked || el.selected)) return false;
    if (ps === "disabled" && !el.disabled) return false;
  }
  return true;
}
function matchComplex(el, sel) {
  const parts = sel.split(/\s+/).filter(Boolean);
  if (!matchCompound(el, parts[parts.length - 1])) return false;
  let cur = el.parentNode;
  for (let i = parts.length - 2; i >= 0; i--) {
    while (cur instanceof Element && !matchCompound(cur, parts[i])) cur = cur.parentNode;
    if (!(cur instanceof Element)) return false;
    cur = cur.parentNode;
  }
  return true;
}

// ---- HTML parsing ---------------------------------------------------------------------------------------
function parseInto(root, html, doc) {
  const stack = [root];
  const re = /<!--[\s\S]*?-->|<!doctype[^>]*>|<\/([a-zA-Z][\w-]*)\s*>|<([a-zA-Z][\w-]*)((?:\s+[^\s=>/]+(?:\s*=\s*(?:"[^"]*"|'[^']*'|[^\s>]+))?)*)\s*(\/?)>|([^<]+|<)/gi;
  let m;
  while ((m = re.exec(html)) !== null) {
    const top = stack[stack.length - 1];
    if (m[1]) {  // close tag
      const t = m[1].toLowerCase();
      for (let i = stack.length - 1; i > 0; i--) {
        if (stack[i].localName === t) { stack.length = i; break; }
      }
    } else if (m[2]) {
      const el = new Element(m[2], doc);
      const are = /([^\s=>/]+)(?:\s*=\s*(?:"([^"]*)"|'([^']*)'|([^\s>]+)))?/g;
      let a;
      while ((a = are.exec(m[3] || "")) !== null) {
        const v = a[2] !== undefined ? a[2] : a[3] !== undefined ? a[3] : a[4] !== undefined ? a[4] : "";
        el.attributes[a[1].toLowerCase()] = decode(v);
      }
      top.appendChild(el);
      if (!VOID.has(el.localName) && !m[4]) stack.push(el);
    } else if (m[5] !== undefined && !/^<!/.test(m[0])) {
      top.appendChild(new Text(decode(m[5])));
    }
  }
}

class Document {
  constructor(html) {
    this.listeners = {};
    this.cookie = "";
    this.documentElement = new Element("html", this);
    parseInto(this.documentElement, html || "<body></body>", this);
    this.body = this.documentElement.querySelector("body") || this.documentElement;
  }
  createElement(t) { return new Element(t, this); }
  createTextNode(t) { return new Text(String(t)); }
  getElementById(id) { return this.documentElement.querySelector(`#${id}`); }
  querySelector(s) { return this.documentElement.querySelector(s); }
  querySelectorAll(s) { return this.documentElement.querySelectorAll(s); }
  addEventListener(type, fn) { (this.listeners[type] = this.listeners[type] || []).push(fn); }
}

// event helpers for tests: set a control's value the way a user does and fire its events
function type(el, value) { el.value = value; el.dispatchEvent({ type: "input" }); el.dispatchEvent({ type: "change" }); }
function choose(select, value) { select.value = value; select.dispatchEvent({ type: "change" }); }

module.exports = { Document, Element, Node, Text, type, choose };
