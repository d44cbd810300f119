// Central dashboard shell (browser wiring of cdb.js): sidenav from /api/dashboard-links, namespace
// selector over the user's workgroups (/api/workgroup/env-info), one persistent iframe for the apps
// under /_/<app>/ with browser <-> iframe URL mirroring and the library.js namespace protocol, home
// page (quick links, recent notebooks, activities, cluster + MI355X GPU charts), contributor
// management, registration flow, namespace-needed and 404 pages.
(function () {
  "use strict";
  const C = window.cdb;
  const $ = (id) => document.getElementById(id);
  const EV = { APP_CONNECTED: "iframe-connected", PARENT_CONNECTED: "parent-connected",
               NAMESPACE_SELECTED: "namespace-selected", ALL_NAMESPACES: "all-namespaces" };
  const state = { env: null, links: {}, options: [], ns: null, frame: null, sync: null };
  const inIframe = window.location !== window.parent.location;

  async function get(path) {
    const r = await fetch(path);
    const d = await r.json();
    if (!r.ok) throw new Error(d.error || r.statusText);
    return d;
  }
  async function send(method, path, body) {
    const r = await fetch(path, { method, headers: { "Content-Type": "application/json" }, body: JSON.stringify(body || {}) });
    const d = await r.json();
    if (!r.ok) throw new Error(d.error || r.statusText);
    return d;
  }

  // ---- router ----------------------------------------------------------------------------------
  const browserUrl = () => location.pathname + location.search + location.hash;
  const router = {
    url: browserUrl,
    navigate(path, params, fragment, replace) {
      const url = path + C.queryString(params || {}) + (fragment !== undefined ? "#" + fragment : "");
      if (url === browserUrl()) return;
      history[replace ? "replaceState" : "pushState"]({}, "", url);
      route(false);
    },
  };
  function go(href, forced) {
    history.pushState({}, "", href);
    route(forced);
  }
  window.addEventListener("popstate", () => route(false));

  // ---- namespace -------------------------------------------------------------------------------
  function postNamespace() {
    const w = state.frame && state.frame.contentWindow;
    if (!w || !state.ns) return;
    if (state.ns.namespace === C.ALL_NAMESPACES) {
      w.postMessage({ type: EV.ALL_NAMESPACES, value: state.options.filter((o) => o.namespace !== C.ALL_NAMESPACES).map((o) => o.namespace) }, location.origin);
    } else {
      w.postMessage({ type: EV.NAMESPACE_SELECTED, value: state.ns.namespace }, location.origin);
    }
  }
  window.addEventListener("message", (ev) => {
    if (ev.origin === location.origin && (ev.data || {}).type === EV.APP_CONNECTED) postNamespace();
  });

  function resolveNamespace() {
    state.options = C.namespaceOptions(state.env.namespaces, browserUrl());
    const queryNs = C.queryParams(location.search).ns;
    const picked = C.pickNamespace(state.options, { queryNs, storedNs: localStorage.getItem(C.storageKey(state.env.user)) });
    const changed = (picked && picked.namespace) !== (state.ns && state.ns.namespace);
    state.ns = picked || null;
    if (picked) localStorage.setItem(C.storageKey(state.env.user), picked.namespace);
    if (picked && queryNs !== picked.namespace) {
      const p = C.queryParams(location.search);
      p.ns = picked.namespace;
      history.replaceState({}, "", location.pathname + C.queryString(p) + location.hash);
    }
    if (changed) postNamespace();
  }

  function selectNamespace(name) {
    const opt = state.options.find((o) => o.namespace === name && !o.disabled);
    if (!opt) return;
    localStorage.setItem(C.storageKey(state.env.user), opt.namespace);
    const p = C.queryParams(location.search);
    p.ns = opt.namespace;
    router.navigate(location.pathname, p, location.hash ? location.hash.slice(1) : undefined, false);
  }

  function renderChrome() {
    const ns = state.ns ? state.ns.namespace : "";
    $("menu").innerHTML = C.renderSidenav(state.links.menuLinks || [], ns, browserUrl(), state.env.platform);
    $("ns").innerHTML = C.renderNamespaceSelector(state.options, state.ns);
    const trigger = $("ns").querySelector("[data-cy-selected-namespace]");
    const menu = $("ns").querySelector(".ns-menu");
    trigger.onclick = () => { if (!trigger.classList.contains("disabled")) menu.hidden = !menu.hidden; };
    menu.querySelectorAll("li[data-ns]").forEach((li) => li.onclick = () => { menu.hidden = true; selectNamespace(li.dataset.ns); });
  }

  document.addEventListener("click", (e) => {
    const a = e.target.closest && e.target.closest("a[data-nav]");
    if (!a || e.ctrlKey || e.metaKey) return;
    e.preventDefault();
    go(a.getAttribute("href"), true);
  });

  // ---- views -----------------------------------------------------------------------------------
  function ensureFrame() {
    if (state.frame && state.frame.isConnected) return state.frame;
    $("content").innerHTML = "";
    state.frame = document.createElement("iframe");
    state.frame.src = "about:blank";
    state.frame.addEventListener("load", () => {
      const w = state.frame.contentWindow;
      if (w) w.postMessage({ type: EV.PARENT_CONNECTED }, location.origin);
    });
    $("content").append(state.frame);
    state.sync = new C.IframeSync(router, () => (state.frame ? state.frame.contentWindow : null),
                                  () => (state.ns ? state.ns.namespace : ""));
    return state.frame;
  }
  setInterval(() => { if (state.sync && state.frame && state.frame.isConnected) state.sync.tick(); }, 100);

  function route(forced) {
    if (!state.env) return;
    resolveNamespace();
    renderChrome();
    const v = C.viewFor(browserUrl());
    if (v.page === "iframe") {
      const f = ensureFrame();
      const src = state.sync.onNavigate(browserUrl(), location.origin, forced);
      if (src !== null) f.src = src;
      return;
    }
    state.frame = null;
    state.sync = null;
    if (v.page === "namespace-needed") $("content").innerHTML = C.renderNamespaceNeeded();
    else if (v.page === "not-found") $("content").innerHTML = C.renderNotFound(v.path);
    else if (v.page === "manage-users") showManageUsers();
    else showHome();
  }

  function chart(points, title) {
    if (!points || !points.length) return `<p>${C.esc(title)}: no data</p>`;
    const w = 300, h = 80, t0 = points[0].timestamp, t1 = points[points.length - 1].timestamp || t0 + 1;
    const vmax = Math.max(1e-9, ...points.map((p) => p.value));
    const path = points.map((p, i) => `${i ? "L" : "M"}${((p.timestamp - t0) / Math.max(1, t1 - t0)) * w},${h - (p.value / vmax) * h}`).join(" ");
    return `<div>${C.esc(title)} <small>(max ${(vmax * 100).toFixed(1)})</small><br><svg width="${w}" height="${h}"><path d="${path}" fill="none" stroke="#1a73e8"/></svg></div>`;
  }

  function showHome() {
    const ns = state.ns && state.ns.namespace !== C.ALL_NAMESPACES ? state.ns.namespace : "";
    const nsq = ns ? C.queryString({ ns }) : "";
    const quick = (state.links.quickLinks || []).map((l) => `<li><a href="${C.esc(C.menuHref(l.link, ns))}" data-nav="1">${C.esc(l.text)}</a> <small>${C.esc(l.desc || "")}</small></li>`).join("");
    const docs = (state.links.documentationItems || []).map((l) => `<li><a href="${C.esc(l.link)}" target="_blank" rel="noopener">${C.esc(l.text)}</a> <small>${C.esc(l.desc || "")}</small></li>`).join("");
    $("content").innerHTML = `<div class="page"><div class="cards">
      <div class="card"><h3>Quick shortcuts</h3><ul>${quick}</ul></div>
      <div class="card"><h3>Recent notebooks${ns ? " in " + C.esc(ns) : ""}</h3><div id="nbs">loading…</div></div>
      <div class="card"><h3>Recent activity${ns ? " in " + C.esc(ns) : ""}</h3><div id="acts">loading…</div></div>
      <div class="card"><h3>Cluster resources</h3><div id="charts">loading…</div></div>
      <div class="card"><h3>Documentation</h3><ul>${docs}</ul></div></div>
      <p><a href="/manage-users${nsq}" data-nav="1">Manage contributors</a></p></div>`;
    if (ns) {
      get(`/jupyter/api/namespaces/${encodeURIComponent(ns)}/notebooks`).then((d) => {
        $("nbs").innerHTML = C.recentNotebooks(d.notebooks).map((nb) =>
          `<div><a href="/notebook/${C.esc(ns)}/${C.esc(nb.name)}/" target="_blank" rel="noopener">${C.esc(nb.name)}</a>
           <small>${C.esc((nb.status || {}).phase)} · ${C.esc((nb.gpus || {}).message || "no GPU")}</small></div>`).join("") || "No notebook servers.";
      }).catch(() => { $("nbs").textContent = "Notebooks app unavailable"; });
      get(`/api/activities/${encodeURIComponent(ns)}`).then((evs) => { $("acts").innerHTML = C.renderActivities(evs); })
        .catch((e) => { $("acts").textContent = e.message; });
    } else {
      $("nbs").textContent = $("acts").textContent = "Select a namespace.";
    }
    Promise.all(["node", "podcpu", "gpu"].map((k) => get(`/api/metrics/${k}?interval=Last60m`).catch(() => null))).then(([n, c, g]) => {
      if (!n) { $("charts").textContent = "Metrics are not available on this cluster."; return; }
      $("charts").innerHTML = chart(n, "Node CPU") + chart(c, "Pod CPU requests") + chart(g, "MI355X GPUs allocated");
    });
  }

  function showManageUsers() {
    const owned = (state.env.namespaces || []).filter((b) => b.role === "owner");
    $("content").innerHTML = `<div class="page"><h2>Manage contributors</h2><p class="err" id="merr"></p>${owned.map((b) => `
      <div class="card"><h3>${C.esc(b.namespace)} <small>(Owner)</small></h3><div data-contribs="${C.esc(b.namespace)}">loading…</div>
      <input data-input="${C.esc(b.namespace)}" placeholder="user@example.com"> <button data-add="${C.esc(b.namespace)}">Add</button></div>`).join("") || "<p>You do not own a namespace.</p>"}
      ${state.env.isClusterAdmin ? '<h3>All namespaces</h3><div id="allns">loading…</div>' : ""}</div>`;
    const box = (ns) => $("content").querySelector(`[data-contribs="${CSS.escape(ns)}"]`);
    const fail = (e) => { $("merr").textContent = e.message; };
    const render = (ns, users) => {
      box(ns).innerHTML = C.renderContributors(ns, users);
      box(ns).querySelectorAll("button[data-rm]").forEach((btn) => btn.onclick = () =>
        send("DELETE", `/api/workgroup/remove-contributor/${encodeURIComponent(ns)}`, { contributor: btn.dataset.rm }).then((u) => render(ns, u)).catch(fail));
    };
    owned.forEach((b) => get(`/api/workgroup/get-contributors/${encodeURIComponent(b.namespace)}`).then((u) => render(b.namespace, u)).catch(fail));
    $("content").querySelectorAll("button[data-add]").forEach((btn) => btn.onclick = () => {
      const ns = btn.dataset.add;
      const input = $("content").querySelector(`[data-input="${CSS.escape(ns)}"]`);
      send("POST", `/api/workgroup/add-contributor/${encodeURIComponent(ns)}`, { contributor: input.value }).then((u) => { input.value = ""; render(ns, u); }).catch(fail);
    });
    if (state.env.isClusterAdmin) {
      get("/api/workgroup/get-all-namespaces").then((rows) => {
        $("allns").innerHTML = `<table><tr><th>Namespace</th><th>Owner</th><th>Contributors</th></tr>${rows.map((r) =>
          `<tr><td>${C.esc(r[0])}</td><td>${C.esc(r[1])}</td><td>${C.esc(r[2])}</td></tr>`).join("")}</table>`;
      }).catch(fail);
    }
  }

  function showRegistration(ex) {
    $("menu").innerHTML = "";
    $("ns").innerHTML = "";
    $("content").innerHTML = `<div class="page"><h2>Welcome, ${C.esc(ex.user)}</h2>
      <p>Create your namespace to start using notebooks on MI355X GPUs.</p>
      <input id="reg-ns" value="${C.esc(C.suggestNamespace(ex.user))}"> <button id="reg">Finish</button> <span class="err" id="rerr"></span></div>`;
    $("reg").onclick = async () => {
      $("reg").disabled = true;
      $("rerr").textContent = "";
      const r = await C.register({ create: (ns) => send("POST", "/api/workgroup/create", { namespace: ns }),
                                   exists: () => get("/api/workgroup/exists") }, $("reg-ns").value);
      $("reg").disabled = false;
      if (r.ok) main();
      else $("rerr").textContent = r.error;
    };
  }

  async function main() {
    if (inIframe) document.body.classList.add("iframed");  // no sidenav/header inside an iframe (no mirror effect)
    try {
      const ex = await get("/api/workgroup/exists");
      if (ex.hasAuth && !ex.hasWorkgroup && ex.registrationFlowAllowed) return showRegistration(ex);
      [state.env, state.links] = await Promise.all([get("/api/workgroup/env-info"), get("/api/dashboard-links").catch(() => ({}))]);
      $("user").textContent = state.env.user;
      $("logout").href = (state.env.platform || {}).logoutUrl || "/logout";
      route(false);
    } catch (e) {
      $("content").innerHTML = `<p class="page err">${C.esc(e.message)}</p>`;
    }
  }
  main();
})();
